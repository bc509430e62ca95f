// Checkpoint archives in the format of the reference's torch::save(model_, path)
// (src/training/tensorboard_trainer_enhanced.h:656-662) — host only, no LibTorch.
//
// torch::save(shared_ptr<nn::Module>) goes through serialize::OutputArchive, which mirrors the module
// tree as TorchScript objects and writes a TorchScript zip archive:
//   <name>/data/<k>            raw little-endian storage of the k-th tensor pickled (stored, 64-byte
//                              aligned)
//   <name>/data.pkl            protocol-2 pickle of the object tree: one "__torch__[.___torch_mangle_N]
//                              Module" object per nn::Module (preorder numbering), its state dict =
//                              parameters, buffers (registration order), then child modules; tensors
//                              are torch._utils._rebuild_tensor_v2(persistent storage id, ...)
//   <name>/code/__torch__[/___torch_mangle_N].py   the TorchScript class declaring __parameters__,
//                              __buffers__ and the typed attributes (what torch::load type-checks)
//   <name>/constants.pkl, version ("3"), byteorder, .data/serialization_id
// The writer emits data.pkl and the class sources byte-identical to LibTorch's (the memo / opcode
// choices of torch::jit::Pickler are reproduced), which tests/test_checkpoint.py checks against an
// archive the reference code wrote in this container; torch::load of the reference reads ours back.
//
// The reader is a data-only pickle interpreter: it understands the opcodes these archives (and
// Python torch.save state dicts) use, builds tensors from persistent storage ids and never calls
// anything named in the file — the equivalent of torch.load(weights_only=True).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <set>
#include <memory>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/cad/cad.h"

namespace cad {
void set_last_error(const std::string& msg);
}

namespace {

struct ArchiveError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

template <class F>
cad_status arch_guard(F&& f) {
    try {
        f();
        return CAD_OK;
    } catch (const std::exception& e) {
        cad::set_last_error(e.what());
        return CAD_ERR_INVALID;
    }
}

// ---------------------------------------------------------------------------------------------
// zip container (stored entries only: LibTorch never compresses tensor records)
// ---------------------------------------------------------------------------------------------
uint32_t crc32_update(uint32_t crc, const uint8_t* p, size_t n) {
    static uint32_t table[256];
    static bool init = false;
    if (!init) {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = c & 1 ? 0xEDB88320u ^ (c >> 1) : c >> 1;
            table[i] = c;
        }
        init = true;
    }
    crc = ~crc;
    for (size_t i = 0; i < n; ++i) crc = table[(crc ^ p[i]) & 0xFF] ^ (crc >> 8);
    return ~crc;
}

void put16(std::string& s, uint16_t v) { s.append(reinterpret_cast<const char*>(&v), 2); }
void put32(std::string& s, uint32_t v) { s.append(reinterpret_cast<const char*>(&v), 4); }

class ZipWriter {
  public:
    explicit ZipWriter(const std::string& path) : path_(path) {
        f_ = std::fopen(path.c_str(), "wb");
        if (!f_) throw ArchiveError("cannot open " + path + " for writing");
    }
    ~ZipWriter() {
        if (f_) std::fclose(f_);
    }
    void add(const std::string& name, const void* data, size_t n) {
        if (n >= 0xFFFFFFFFull || pos_ >= 0xFFFFFFFFull) throw ArchiveError("archive larger than 4 GB (zip64) is not supported");
        const uint32_t crc = crc32_update(0, static_cast<const uint8_t*>(data), n);
        // pad the local extra field ("FB" block, as LibTorch does) so the data starts 64-byte aligned
        const size_t hdr = 30 + name.size() + 4;
        const size_t pad = (64 - (pos_ + hdr) % 64) % 64;
        const uint64_t off = pos_;
        std::string h;
        put32(h, 0x04034b50); put16(h, 20); put16(h, 0); put16(h, 0); put16(h, 0); put16(h, 0x21);
        put32(h, crc); put32(h, (uint32_t)n); put32(h, (uint32_t)n);
        put16(h, (uint16_t)name.size()); put16(h, (uint16_t)(4 + pad));
        h += name;
        put16(h, 0x4246); put16(h, (uint16_t)pad);
        h.append(pad, 'Z');
        write(h.data(), h.size());
        ents_.push_back({name, crc, (uint32_t)n, (uint32_t)off});
        write(data, n);
    }
    void finish() {
        const uint64_t cd = pos_;
        for (const auto& e : ents_) {
            std::string h;
            put32(h, 0x02014b50); put16(h, 20); put16(h, 20); put16(h, 0); put16(h, 0); put16(h, 0); put16(h, 0x21);
            put32(h, e.crc); put32(h, e.size); put32(h, e.size);
            put16(h, (uint16_t)e.name.size()); put16(h, 0); put16(h, 0); put16(h, 0); put16(h, 0); put32(h, 0);
            put32(h, e.off);
            h += e.name;
            write(h.data(), h.size());
        }
        const uint64_t cd_size = pos_ - cd;
        if (pos_ >= 0xFFFFFFFFull || ents_.size() >= 0xFFFF) throw ArchiveError("archive too large for a non-zip64 directory");
        std::string h;
        put32(h, 0x06054b50); put16(h, 0); put16(h, 0); put16(h, (uint16_t)ents_.size()); put16(h, (uint16_t)ents_.size());
        put32(h, (uint32_t)cd_size); put32(h, (uint32_t)cd); put16(h, 0);
        write(h.data(), h.size());
        if (std::fclose(f_) != 0) { f_ = nullptr; throw ArchiveError("write failed: " + path_); }
        f_ = nullptr;
    }

  private:
    struct Ent {
        std::string name;
        uint32_t crc, size, off;
    };
    void write(const void* p, size_t n) {
        if (n && std::fwrite(p, 1, n, f_) != n) throw ArchiveError("write failed: " + path_);
        pos_ += n;
    }
    std::string path_;
    FILE* f_ = nullptr;
    uint64_t pos_ = 0;
    std::vector<Ent> ents_;
};

// ---------------------------------------------------------------------------------------------
// pickle writer reproducing torch::jit::Pickler's output for module state
// ---------------------------------------------------------------------------------------------
class Pickler {
  public:
    std::string out;
    void op(uint8_t c) { out.push_back((char)c); }
    void put() {
        const uint32_t id = memo_++;
        if (id < 256) { op('q'); op((uint8_t)id); }
        else { op('r'); put32(out, id); }
    }
    void get(uint32_t id) {
        if (id < 256) { op('h'); op((uint8_t)id); }
        else { op('j'); put32(out, id); }
    }
    void str(const std::string& s) {
        auto it = strs_.find(s);
        if (it != strs_.end()) return get(it->second);
        op('X'); put32(out, (uint32_t)s.size()); out += s;
        strs_[s] = memo_;
        put();
    }
    void global(const std::string& mod, const std::string& name) {
        const std::string k = mod + "\n" + name + "\n";
        auto it = globals_.find(k);
        if (it != globals_.end()) return get(it->second);
        op('c'); out += k;
        globals_[k] = memo_;
        put();
    }
    void integer(int64_t n) {
        if (n >= 0 && n <= 0xFF) { op('K'); op((uint8_t)n); }
        else if (n >= 0 && n <= 0xFFFF) { op('M'); put16(out, (uint16_t)n); }
        else if (n >= INT32_MIN && n <= INT32_MAX) { op('J'); put32(out, (uint32_t)(int32_t)n); }
        else { op(0x8a); op(8); out.append(reinterpret_cast<const char*>(&n), 8); }
    }

  private:
    uint32_t memo_ = 0;
    std::map<std::string, uint32_t> strs_, globals_;
};

const char* storage_name(int dtype) {
    switch (dtype) {
        case CAD_DTYPE_F32: return "FloatStorage";
        case CAD_DTYPE_I64: return "LongStorage";
        case CAD_DTYPE_F64: return "DoubleStorage";
        case CAD_DTYPE_F16: return "HalfStorage";
        case CAD_DTYPE_BF16: return "BFloat16Storage";
        case CAD_DTYPE_I32: return "IntStorage";
        default: throw ArchiveError("unsupported dtype code " + std::to_string(dtype));
    }
}
int dtype_bytes(int dtype) {
    switch (dtype) {
        case CAD_DTYPE_F32: case CAD_DTYPE_I32: return 4;
        case CAD_DTYPE_I64: case CAD_DTYPE_F64: return 8;
        case CAD_DTYPE_F16: case CAD_DTYPE_BF16: return 2;
        default: throw ArchiveError("unsupported dtype code " + std::to_string(dtype));
    }
}

struct ModNode {
    std::string name;   // attribute name in the parent
    std::vector<const cad_archive_entry*> params, buffers;
    std::vector<std::unique_ptr<ModNode>> children;
    int cls = -1;       // -1 = root "__torch__.Module", else ___torch_mangle_<cls>
    ModNode* child(const std::string& n) {
        for (auto& c : children)
            if (c->name == n) return c.get();
        children.push_back(std::make_unique<ModNode>());
        children.back()->name = n;
        return children.back().get();
    }
};

std::string class_path(const ModNode& m) {
    return m.cls < 0 ? std::string("__torch__") : "__torch__.___torch_mangle_" + std::to_string(m.cls);
}

void number(ModNode& m, int& next) {
    for (auto& c : m.children) {
        c->cls = next++;
        number(*c, next);
    }
}

struct ArchiveOut {
    ZipWriter& zip;
    std::string prefix;
    Pickler pk;
    int next_key = 0;
    std::map<int, std::pair<std::string, std::string>> code;   // class number -> (file, source)

    void tensor(const cad_archive_entry& e, bool requires_grad) {
        int64_t numel = 1;
        for (int i = 0; i < e.ndim; ++i) numel *= e.shape[i];
        const std::string key = std::to_string(next_key++);
        zip.add(prefix + "/data/" + key, e.data, (size_t)numel * dtype_bytes(e.dtype));
        pk.global("torch._utils", "_rebuild_tensor_v2");
        pk.op('(');
        pk.op('(');
        pk.str("storage");
        pk.global("torch", storage_name(e.dtype));
        pk.str(key);
        pk.str("cpu");
        pk.integer(numel);
        pk.op('t');
        pk.op('Q');
        pk.put();
        pk.integer(0);
        pk.op('(');
        for (int i = 0; i < e.ndim; ++i) pk.integer(e.shape[i]);
        pk.op('t');
        pk.op('(');
        int64_t stride = 1;
        std::vector<int64_t> st((size_t)e.ndim);
        for (int i = e.ndim - 1; i >= 0; --i) { st[(size_t)i] = stride; stride *= e.shape[i]; }
        for (int i = 0; i < e.ndim; ++i) pk.integer(st[(size_t)i]);
        pk.op('t');
        pk.op(requires_grad ? 0x88 : 0x89);
        pk.global("collections", "OrderedDict");
        pk.op(')');
        pk.op('R');
        pk.op('t');
        pk.op('R');
        pk.put();
    }

    void module(const ModNode& m, bool root) {
        const std::string cp = class_path(m);
        pk.global(cp, "Module");
        pk.op(')');
        pk.op(0x81);   // NEWOBJ
        pk.op('}');
        pk.op('(');
        for (auto* e : m.params) { pk.str(leaf(e->name)); tensor(*e, true); }
        for (auto* e : m.buffers) { pk.str(leaf(e->name)); tensor(*e, false); }
        for (auto& c : m.children) { pk.str(c->name); module(*c, false); }
        pk.op('u');
        pk.op('b');
        if (root) pk.put();
        // the TorchScript class declaring this module's attributes
        std::string src = "class Module(Module):\n  __parameters__ = [";
        for (auto* e : m.params) src += "\"" + leaf(e->name) + "\", ";
        src += "]\n  __buffers__ = [";
        for (auto* e : m.buffers) src += "\"" + leaf(e->name) + "\", ";
        src += "]\n";
        for (auto* e : m.params) src += "  " + leaf(e->name) + " : Tensor\n";
        for (auto* e : m.buffers) src += "  " + leaf(e->name) + " : Tensor\n";
        for (auto& c : m.children) src += "  " + c->name + " : " + class_path(*c) + ".Module\n";
        const std::string file = m.cls < 0 ? "code/__torch__.py" : "code/__torch__/___torch_mangle_" + std::to_string(m.cls) + ".py";
        code[m.cls] = {file, src};
    }
    static std::string leaf(const char* dotted) {
        const char* p = std::strrchr(dotted, '.');
        return p ? std::string(p + 1) : std::string(dotted);
    }
};

// ---------------------------------------------------------------------------------------------
// reader
// ---------------------------------------------------------------------------------------------
struct ZipEntry {
    uint64_t data_off, size;
    uint16_t method;
};

uint16_t rd16(const uint8_t* p) { uint16_t v; std::memcpy(&v, p, 2); return v; }
uint32_t rd32(const uint8_t* p) { uint32_t v; std::memcpy(&v, p, 4); return v; }

struct Value;
using VPtr = std::shared_ptr<Value>;
struct Value {
    enum Kind { None, Bool, Int, Float, Str, Tuple, List, Dict, Global, Object, Storage, Tensor, Mark, Opaque } kind = None;
    int64_t i = 0;
    double d = 0;
    std::string s, s2;                               // Str / Global (module, name) / Object class
    std::vector<VPtr> items;                         // Tuple / List
    std::vector<std::pair<VPtr, VPtr>> dict;         // Dict / Object state
    // Storage: s = key, i = dtype; Tensor: storage in items[0], i = offset, sizes/strides
    std::vector<int64_t> sizes, strides;
};

VPtr mk(Value::Kind k) {
    auto v = std::make_shared<Value>();
    v->kind = k;
    return v;
}

int dtype_of_storage(const std::string& name) {
    if (name == "FloatStorage") return CAD_DTYPE_F32;
    if (name == "LongStorage") return CAD_DTYPE_I64;
    if (name == "DoubleStorage") return CAD_DTYPE_F64;
    if (name == "HalfStorage") return CAD_DTYPE_F16;
    if (name == "BFloat16Storage") return CAD_DTYPE_BF16;
    if (name == "IntStorage") return CAD_DTYPE_I32;
    throw ArchiveError("unsupported storage type torch." + name);
}

class Unpickler {
  public:
    Unpickler(const std::string& b) : b_(b) {}
    VPtr run() {
        for (;;) {
            const uint8_t c = byte();
            switch (c) {
                case 0x80: byte(); break;                                  // PROTO
                case 0x95: take(8); break;                                 // FRAME
                case '(': push(mk(Value::Mark)); break;
                case 'N': push(mk(Value::None)); break;
                case 0x88: case 0x89: { auto v = mk(Value::Bool); v->i = c == 0x88; push(v); break; }
                case 'K': { auto v = mk(Value::Int); v->i = byte(); push(v); break; }
                case 'M': { auto v = mk(Value::Int); v->i = rd16(take(2)); push(v); break; }
                case 'J': { auto v = mk(Value::Int); v->i = (int32_t)rd32(take(4)); push(v); break; }
                case 0x8a: {                                               // LONG1
                    const int n = byte();
                    if (n > 8) throw ArchiveError("pickle: integer wider than 64 bits");
                    const uint8_t* p = take((size_t)n);
                    int64_t v = 0;
                    for (int k = n - 1; k >= 0; --k) v = (v << 8) | p[k];
                    if (n > 0 && n < 8 && (p[n - 1] & 0x80)) v -= (int64_t)1 << (8 * n);
                    auto x = mk(Value::Int); x->i = v; push(x); break;
                }
                case 'G': {                                                // BINFLOAT (big-endian)
                    const uint8_t* p = take(8);
                    uint64_t u = 0;
                    for (int k = 0; k < 8; ++k) u = (u << 8) | p[k];
                    auto v = mk(Value::Float); std::memcpy(&v->d, &u, 8); push(v); break;
                }
                case 'X': { const uint32_t n = rd32(take(4)); push_str(n); break; }
                case 0x8c: { const uint32_t n = byte(); push_str(n); break; }
                case 0x8d: { uint64_t n; std::memcpy(&n, take(8), 8); push_str(n); break; }
                case 'B': { const uint32_t n = rd32(take(4)); push_str(n); break; }
                case 'C': { const uint32_t n = byte(); push_str(n); break; }
                case 'c': {                                                // GLOBAL
                    auto v = mk(Value::Global);
                    v->s = line();
                    v->s2 = line();
                    push(v);
                    break;
                }
                case 0x93: {                                               // STACK_GLOBAL
                    auto name = pop(), mod = pop();
                    auto v = mk(Value::Global); v->s = mod->s; v->s2 = name->s; push(v); break;
                }
                case 'q': memo_[byte()] = top(); break;
                case 'r': memo_[rd32(take(4))] = top(); break;
                case 0x94: memo_[(uint32_t)memo_.size()] = top(); break;   // MEMOIZE
                case 'h': push(memo(byte())); break;
                case 'j': push(memo(rd32(take(4)))); break;
                case ')': push(mk(Value::Tuple)); break;
                case ']': push(mk(Value::List)); break;
                case '}': push(mk(Value::Dict)); break;
                case 't': { auto v = mk(Value::Tuple); v->items = pop_mark(); push(v); break; }
                case 0x85: case 0x86: case 0x87: {
                    const int n = c - 0x84;
                    auto v = mk(Value::Tuple);
                    v->items.resize((size_t)n);
                    for (int k = n - 1; k >= 0; --k) v->items[(size_t)k] = pop();
                    push(v);
                    break;
                }
                case 'a': { auto x = pop(); list(top())->items.push_back(x); break; }
                case 'e': { auto xs = pop_mark(); auto& l = list(top())->items; l.insert(l.end(), xs.begin(), xs.end()); break; }
                case 's': { auto v = pop(), k = pop(); dict(top())->dict.push_back({k, v}); break; }
                case 'u': {
                    auto xs = pop_mark();
                    if (xs.size() % 2) throw ArchiveError("pickle: odd SETITEMS");
                    auto d = dict(top());
                    for (size_t k = 0; k < xs.size(); k += 2) d->dict.push_back({xs[k], xs[k + 1]});
                    break;
                }
                case 'Q': push(persistent(pop())); break;                  // BINPERSID
                case 'R': { auto args = pop(), fn = pop(); push(reduce(fn, args)); break; }
                case 0x81: {                                               // NEWOBJ: cls(*args)
                    pop();
                    auto cls = pop();
                    if (cls->kind != Value::Global) throw ArchiveError("pickle: NEWOBJ of a non-class");
                    auto o = mk(Value::Object);
                    o->s = cls->s + "." + cls->s2;
                    push(o);
                    break;
                }
                case 'b': {                                                // BUILD: obj.__setstate__(state)
                    auto state = pop();
                    auto o = top();
                    if (o->kind == Value::Object && state->kind == Value::Dict) o->dict = state->dict;
                    break;
                }
                case '.': return pop();
                default: {
                    char buf[64];
                    std::snprintf(buf, sizeof buf, "pickle: unsupported opcode 0x%02x at %zu", c, pos_ - 1);
                    throw ArchiveError(buf);
                }
            }
        }
    }

  private:
    const std::string& b_;
    size_t pos_ = 0;
    std::vector<VPtr> st_;
    std::map<uint32_t, VPtr> memo_;

    uint8_t byte() { return *take(1); }
    const uint8_t* take(size_t n) {
        if (n > b_.size() - pos_) throw ArchiveError("pickle: truncated");   // (no pos_ + n wrap)
        const uint8_t* p = reinterpret_cast<const uint8_t*>(b_.data()) + pos_;
        pos_ += n;
        return p;
    }
    std::string line() {
        const size_t e = b_.find('\n', pos_);
        if (e == std::string::npos) throw ArchiveError("pickle: truncated GLOBAL");
        std::string s = b_.substr(pos_, e - pos_);
        pos_ = e + 1;
        return s;
    }
    void push_str(uint64_t n) {
        auto v = mk(Value::Str);
        v->s.assign(reinterpret_cast<const char*>(take((size_t)n)), (size_t)n);
        push(v);
    }
    void push(VPtr v) { st_.push_back(std::move(v)); }
    VPtr pop() {
        if (st_.empty()) throw ArchiveError("pickle: stack underflow");
        auto v = st_.back();
        st_.pop_back();
        return v;
    }
    VPtr top() {
        if (st_.empty()) throw ArchiveError("pickle: stack underflow");
        return st_.back();
    }
    VPtr memo(uint32_t id) {
        auto it = memo_.find(id);
        if (it == memo_.end()) throw ArchiveError("pickle: bad memo reference");
        return it->second;
    }
    std::vector<VPtr> pop_mark() {
        std::vector<VPtr> xs;
        for (;;) {
            auto v = pop();
            if (v->kind == Value::Mark) break;
            xs.push_back(v);
        }
        return std::vector<VPtr>(xs.rbegin(), xs.rend());
    }
    static VPtr list(VPtr v) {
        if (v->kind != Value::List) throw ArchiveError("pickle: APPEND to a non-list");
        return v;
    }
    static VPtr dict(VPtr v) {
        if (v->kind != Value::Dict) throw ArchiveError("pickle: SETITEM on a non-dict");
        return v;
    }
    static VPtr persistent(VPtr pid) {
        // ('storage', <torch.XStorage>, key, location, numel)
        if (pid->kind != Value::Tuple || pid->items.size() < 5 || pid->items[0]->s != "storage" ||
            pid->items[1]->kind != Value::Global)
            throw ArchiveError("pickle: unsupported persistent id");
        auto s = mk(Value::Storage);
        s->s = pid->items[2]->s;
        s->i = dtype_of_storage(pid->items[1]->s2);
        return s;
    }
    static std::vector<int64_t> ints(const VPtr& t) {
        std::vector<int64_t> v;
        for (auto& x : t->items) {
            if (x->kind != Value::Int) throw ArchiveError("pickle: expected an int tuple");
            v.push_back(x->i);
        }
        return v;
    }
    static VPtr reduce(const VPtr& fn, const VPtr& args) {
        if (fn->kind != Value::Global) throw ArchiveError("pickle: REDUCE of a non-callable");
        const std::string f = fn->s + "." + fn->s2;
        if (f == "torch._utils._rebuild_tensor_v2" || f == "torch._utils._rebuild_tensor") {
            if (args->items.size() < 4 || args->items[0]->kind != Value::Storage)
                throw ArchiveError("pickle: malformed _rebuild_tensor_v2");
            auto t = mk(Value::Tensor);
            t->items = {args->items[0]};
            t->i = args->items[1]->i;
            t->sizes = ints(args->items[2]);
            t->strides = ints(args->items[3]);
            return t;
        }
        if (f == "torch._utils._rebuild_parameter" || f == "torch._utils._rebuild_parameter_with_state") {
            if (args->items.empty() || args->items[0]->kind != Value::Tensor) throw ArchiveError("pickle: malformed parameter");
            return args->items[0];
        }
        if (f == "collections.OrderedDict") return mk(Value::Dict);
        return mk(Value::Opaque);   // anything else is data we do not need; nothing is called
    }
};

}  // namespace

struct cad_archive {
    std::string path, prefix;
    std::map<std::string, ZipEntry> entries;
    struct T {
        std::string name, key;
        int dtype;
        int64_t offset;
        std::vector<int64_t> sizes;
    };
    std::vector<T> tensors;
};

namespace {

std::string read_range(FILE* f, uint64_t off, uint64_t n) {
    std::string s((size_t)n, '\0');
    if (std::fseek(f, (long)off, SEEK_SET) != 0 || (n && std::fread(&s[0], 1, (size_t)n, f) != n))
        throw ArchiveError("read failed");
    return s;
}

// The module tree of an archive is a few levels deep; anything deeper (or a dict that contains
// itself through the memo) is malformed input, not a checkpoint.
constexpr int kMaxDepth = 64;
constexpr int64_t kMaxNumel = (int64_t)1 << 40;

// Total nodes one traversal may visit: a memoised dict reused k times per level is a DAG, not a cycle,
// and would otherwise be walked k^depth times.
constexpr int64_t kMaxVisits = (int64_t)1 << 20;

void collect(const VPtr& v, const std::string& prefix, cad_archive& a, std::set<const Value*>& open, int depth,
             int64_t& visits) {
    if (depth > kMaxDepth) throw ArchiveError("pickle: module tree nested too deeply");
    if (++visits > kMaxVisits) throw ArchiveError("pickle: module tree too large (shared sub-trees)");
    if (v->kind == Value::Tensor) {
        if (v->items.empty() || v->items[0]->kind != Value::Storage) throw ArchiveError("tensor '" + prefix + "' has no storage");
        if (v->strides.size() != v->sizes.size()) throw ArchiveError("tensor '" + prefix + "': sizes and strides differ in rank");
        if (v->i < 0) throw ArchiveError("tensor '" + prefix + "': negative storage offset");
        cad_archive::T t;
        t.name = prefix;
        t.key = v->items[0]->s;
        t.dtype = (int)v->items[0]->i;
        t.offset = v->i;
        t.sizes = v->sizes;
        int64_t expect = 1;
        for (int k = (int)t.sizes.size() - 1; k >= 0; --k) {
            const int64_t n = t.sizes[(size_t)k];
            if (n < 0 || n > kMaxNumel) throw ArchiveError("tensor '" + prefix + "': bad size");
            if (n != 1 && v->strides[(size_t)k] != expect)
                throw ArchiveError("tensor '" + prefix + "' is not contiguous");
            if (n > 0 && expect > kMaxNumel / n) throw ArchiveError("tensor '" + prefix + "': too many elements");
            expect *= n;
        }
        if (t.offset > kMaxNumel) throw ArchiveError("tensor '" + prefix + "': bad storage offset");
        a.tensors.push_back(std::move(t));
        return;
    }
    if (v->kind == Value::Object || v->kind == Value::Dict) {
        if (!open.insert(v.get()).second) throw ArchiveError("pickle: self-referencing module tree");
        for (auto& kv : v->dict) {
            if (kv.first->kind != Value::Str) continue;
            collect(kv.second, prefix.empty() ? kv.first->s : prefix + "." + kv.first->s, a, open, depth + 1, visits);
        }
        open.erase(v.get());
    }
}

}  // namespace

extern "C" {

cad_status cad_archive_write(const char* path, const cad_archive_entry* entries, int n) {
    return arch_guard([&] {
        if (!path || (n > 0 && !entries) || n < 0) throw ArchiveError("bad arguments");
        // the module tree, children in first-appearance order (= registration order for entries
        // given in named_parameters() order with empty submodules placed where they are registered)
        ModNode root;
        for (int k = 0; k < n; ++k) {
            const cad_archive_entry& e = entries[k];
            if (!e.name || !*e.name) throw ArchiveError("entry without a name");
            if (e.kind < 0 || e.kind > 2) throw ArchiveError(std::string("bad entry kind for ") + e.name);
            if (e.kind != 2) {
                if (!e.data || e.ndim < 0 || e.ndim > 8) throw ArchiveError(std::string("bad tensor entry ") + e.name);
                dtype_bytes(e.dtype);
            }
            std::string name(e.name);
            ModNode* m = &root;
            size_t start = 0;
            for (;;) {
                const size_t dot = name.find('.', start);
                if (dot == std::string::npos) break;
                m = m->child(name.substr(start, dot - start));
                start = dot + 1;
            }
            const std::string leaf = name.substr(start);
            if (e.kind == 2) m->child(leaf);
            else if (e.kind == 0) m->params.push_back(&e);
            else m->buffers.push_back(&e);
        }
        int next = 0;
        number(root, next);
        std::string base(path);
        const size_t sl = base.find_last_of('/');
        std::string prefix = sl == std::string::npos ? base : base.substr(sl + 1);
        const size_t dot = prefix.find_last_of('.');
        if (dot != std::string::npos && dot > 0) prefix = prefix.substr(0, dot);
        if (prefix.empty()) prefix = "archive";
        ZipWriter zip(path);
        ArchiveOut ao{zip, prefix, Pickler{}, 0, {}};
        ao.pk.op(0x80);
        ao.pk.op(2);
        ao.module(root, true);
        ao.pk.op('.');
        zip.add(prefix + "/data.pkl", ao.pk.out.data(), ao.pk.out.size());
        // class sources in numbering order (root first)
        for (auto& kv : ao.code) zip.add(prefix + "/" + kv.second.first, kv.second.second.data(), kv.second.second.size());
        const char constants[] = "\x80\x02).";
        zip.add(prefix + "/constants.pkl", constants, 4);
        zip.add(prefix + "/version", "3\n", 2);
        zip.add(prefix + "/byteorder", "little", 6);
        std::random_device rd;
        std::string sid;
        for (int k = 0; k < 40; ++k) sid.push_back((char)('0' + rd() % 10));
        zip.add(prefix + "/.data/serialization_id", sid.data(), sid.size());
        zip.finish();
    });
}

cad_status cad_archive_open(const char* path, cad_archive** out) {
    return arch_guard([&] {
        if (!path || !out) throw ArchiveError("bad arguments");
        std::unique_ptr<FILE, int (*)(FILE*)> f(std::fopen(path, "rb"), std::fclose);
        if (!f) throw ArchiveError(std::string("cannot open ") + path);
        std::fseek(f.get(), 0, SEEK_END);
        const long size = std::ftell(f.get());
        if (size < 22) throw ArchiveError(std::string("not a zip archive: ") + path);
        const long tail = std::min<long>(size, 22 + 65535);
        const std::string t = read_range(f.get(), (uint64_t)(size - tail), (uint64_t)tail);
        long eocd = -1;
        for (long k = tail - 22; k >= 0; --k)
            if (rd32(reinterpret_cast<const uint8_t*>(t.data()) + k) == 0x06054b50) { eocd = k; break; }
        if (eocd < 0) throw ArchiveError(std::string("not a zip archive (no end of central directory): ") + path);
        const uint8_t* e = reinterpret_cast<const uint8_t*>(t.data()) + eocd;
        const uint16_t count = rd16(e + 10);
        const uint32_t cd_size = rd32(e + 12), cd_off = rd32(e + 16);
        if (cd_off == 0xFFFFFFFFu || count == 0xFFFF) throw ArchiveError("zip64 archives are not supported");
        const std::string cd = read_range(f.get(), cd_off, cd_size);
        auto a = std::make_unique<cad_archive>();
        a->path = path;
        size_t p = 0;
        for (int k = 0; k < count; ++k) {
            if (p + 46 > cd.size()) throw ArchiveError("truncated central directory");
            const uint8_t* h = reinterpret_cast<const uint8_t*>(cd.data()) + p;
            if (rd32(h) != 0x02014b50) throw ArchiveError("bad central directory entry");
            const uint16_t method = rd16(h + 10);
            const uint32_t csize = rd32(h + 20), usize = rd32(h + 24);
            const uint16_t nlen = rd16(h + 28), xlen = rd16(h + 30), clen = rd16(h + 32);
            const uint32_t loff = rd32(h + 42);
            std::string name = cd.substr(p + 46, nlen);
            p += 46 + nlen + xlen + clen;
            if (csize == 0xFFFFFFFFu || usize == 0xFFFFFFFFu || loff == 0xFFFFFFFFu)
                throw ArchiveError("zip64 archives are not supported");
            const std::string lh = read_range(f.get(), loff, 30);
            const uint8_t* l = reinterpret_cast<const uint8_t*>(lh.data());
            if (rd32(l) != 0x04034b50) throw ArchiveError("bad local header for " + name);
            a->entries[name] = ZipEntry{(uint64_t)loff + 30 + rd16(l + 26) + rd16(l + 28), usize, method};
            if (a->prefix.empty()) a->prefix = name.substr(0, name.find('/'));
        }
        auto pk = a->entries.find(a->prefix + "/data.pkl");
        if (pk == a->entries.end()) throw ArchiveError(std::string("no data.pkl in ") + path + " (not a torch::save archive)");
        if (pk->second.method != 0) throw ArchiveError("compressed data.pkl is not supported");
        const std::string pkl = read_range(f.get(), pk->second.data_off, pk->second.size);
        Unpickler up(pkl);
        std::set<const Value*> open;
        int64_t visits = 0;
        collect(up.run(), "", *a, open, 0, visits);
        for (auto& t : a->tensors) {
            auto it = a->entries.find(a->prefix + "/data/" + t.key);
            if (it == a->entries.end()) throw ArchiveError("missing storage record data/" + t.key);
            if (it->second.method != 0) throw ArchiveError("compressed storage record data/" + t.key);
            int64_t numel = 1;
            for (auto s : t.sizes) numel *= s;
            if ((uint64_t)(t.offset + numel) * dtype_bytes(t.dtype) > it->second.size)
                throw ArchiveError("storage record data/" + t.key + " is too small for '" + t.name + "'");
        }
        *out = a.release();
    });
}

void cad_archive_close(cad_archive* a) { delete a; }

int cad_archive_count(const cad_archive* a) { return a ? (int)a->tensors.size() : -1; }

int cad_archive_find(const cad_archive* a, const char* name) {
    if (!a || !name) return -1;
    for (size_t k = 0; k < a->tensors.size(); ++k)
        if (a->tensors[k].name == name) return (int)k;
    return -1;
}

cad_status cad_archive_info(const cad_archive* a, int i, const char** name, int* dtype, int* ndim, int64_t shape[8]) {
    return arch_guard([&] {
        if (!a || i < 0 || i >= (int)a->tensors.size()) throw ArchiveError("tensor index out of range");
        const auto& t = a->tensors[(size_t)i];
        if (t.sizes.size() > 8) throw ArchiveError("tensor rank > 8");
        if (name) *name = t.name.c_str();
        if (dtype) *dtype = t.dtype;
        if (ndim) *ndim = (int)t.sizes.size();
        if (shape)
            for (size_t k = 0; k < 8; ++k) shape[k] = k < t.sizes.size() ? t.sizes[k] : 1;
    });
}

cad_status cad_archive_read(const cad_archive* a, int i, void* dst, int64_t bytes) {
    return arch_guard([&] {
        if (!a || i < 0 || i >= (int)a->tensors.size() || !dst) throw ArchiveError("bad arguments");
        const auto& t = a->tensors[(size_t)i];
        int64_t numel = 1;
        for (auto s : t.sizes) numel *= s;
        const int64_t nb = numel * dtype_bytes(t.dtype);
        if (bytes != nb) throw ArchiveError("'" + t.name + "' holds " + std::to_string(nb) + " bytes");
        const ZipEntry& z = a->entries.at(a->prefix + "/data/" + t.key);
        std::unique_ptr<FILE, int (*)(FILE*)> f(std::fopen(a->path.c_str(), "rb"), std::fclose);
        if (!f) throw ArchiveError("cannot reopen " + a->path);
        const std::string s = read_range(f.get(), z.data_off + (uint64_t)t.offset * dtype_bytes(t.dtype), (uint64_t)nb);
        std::memcpy(dst, s.data(), (size_t)nb);
    });
}

}  // extern "C"

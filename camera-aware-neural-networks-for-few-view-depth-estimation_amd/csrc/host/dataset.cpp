// The loader side of the data path: SunRGBDLoader's manifest, file discovery
// and decoding (src/data/sunrgbd_loader.cpp) on the host, and a prefetch ring that decodes upcoming
// batches on worker threads into pinned buffers, uploads them on a copy stream and hands them to the
// device batcher (cad_batcher_assemble: resize + augmentation on the GPU) — so the step never waits
// on the host for its next batch.
//
//   manifest    loadManifest :39-78        "images"[] entries with valid == true, an allowed
//                                           sensor_type, and <path>/intrinsics.txt present, in order
//   files       findRGBImage :80-90         first .jpg/.png under <path>/image (we: first in name order;
//               findDepthImage :92-102      the reference takes directory-iteration order) and .png
//                                           under <path>/depth; PNM (.ppm/.pgm) accepted as raw formats
//   decoding    loadRGB :221-233            cv::imread(IMREAD_COLOR) -> RGB u8 (gray replicated, alpha
//                                           dropped, 16-bit reduced to its high byte)
//               loadDepth :235-259          cv::imread(IMREAD_UNCHANGED): 16-bit -> u16 * 1/1000 m,
//                                           8-bit -> value as metres (convertTo CV_32F, scale 1)
//               loadIntrinsics :261-275     9 whitespace-separated floats, row-major
// PNG is decoded here (zlib inflate + the five scanline filters, non-interlaced, 8/16-bit gray /
// gray+alpha / RGB / RGBA and 8-bit palette); JPEG by jpeg.cpp, which restates libjpeg-turbo's default
// decompression (sequential Huffman, ISLOW IDCT, fancy upsampling, jdcolor.c tables) bit for bit.
//
// The manifest is JSON (the reference uses nlohmann::json, absent here): a small RFC 8259 parser.
#include <hip/hip_runtime.h>
#include <zlib.h>

#include <algorithm>
#include <cctype>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <filesystem>
#include <fstream>
#include <memory>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/cad/cad.h"
#include "jpeg.hpp"

namespace cad {
void set_last_error(const std::string& msg);
}

namespace fs = std::filesystem;

namespace {

struct DataError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

template <class F>
cad_status data_guard(F&& f) {
    try {
        f();
        return CAD_OK;
    } catch (const std::exception& e) {
        cad::set_last_error(e.what());
        return CAD_ERR_INVALID;
    }
}

// ---------------------------------------------------------------------------------------------
// JSON
// ---------------------------------------------------------------------------------------------
struct Json {
    enum Type { Null, Bool, Num, Str, Arr, Obj } t = Null;
    bool b = false;
    double n = 0;
    std::string s;
    std::vector<Json> a;
    std::vector<std::pair<std::string, Json>> o;
    const Json* get(const std::string& k) const {
        if (t != Obj) return nullptr;
        for (auto& kv : o)
            if (kv.first == k) return &kv.second;
        return nullptr;
    }
};

class JsonParser {
  public:
    JsonParser(const std::string& text, const std::string& what) : p_(text.data()), b_(text.data()), e_(text.data() + text.size()), what_(what) {}
    Json parse() {
        Json v = value(0);
        ws();
        if (p_ != e_) fail("trailing characters");
        return v;
    }

  private:
    const char *p_, *b_, *e_;
    std::string what_;
    [[noreturn]] void fail(const std::string& m) const {
        throw DataError(what_ + ": JSON error at byte " + std::to_string(p_ - b_) + ": " + m);
    }
    void ws() {
        while (p_ < e_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) ++p_;
    }
    bool lit(const char* w) {
        const size_t n = std::strlen(w);
        if ((size_t)(e_ - p_) >= n && std::memcmp(p_, w, n) == 0) { p_ += n; return true; }
        return false;
    }
    Json value(int depth) {
        if (depth > 256) fail("nesting too deep");
        ws();
        if (p_ >= e_) fail("unexpected end");
        Json v;
        const char c = *p_;
        if (c == '{') {
            v.t = Json::Obj;
            ++p_;
            ws();
            if (p_ < e_ && *p_ == '}') { ++p_; return v; }
            for (;;) {
                ws();
                if (p_ >= e_ || *p_ != '"') fail("expected a key");
                std::string k = str();
                ws();
                if (p_ >= e_ || *p_ != ':') fail("expected ':'");
                ++p_;
                v.o.emplace_back(std::move(k), value(depth + 1));
                ws();
                if (p_ < e_ && *p_ == ',') { ++p_; continue; }
                if (p_ < e_ && *p_ == '}') { ++p_; return v; }
                fail("expected ',' or '}'");
            }
        }
        if (c == '[') {
            v.t = Json::Arr;
            ++p_;
            ws();
            if (p_ < e_ && *p_ == ']') { ++p_; return v; }
            for (;;) {
                v.a.push_back(value(depth + 1));
                ws();
                if (p_ < e_ && *p_ == ',') { ++p_; continue; }
                if (p_ < e_ && *p_ == ']') { ++p_; return v; }
                fail("expected ',' or ']'");
            }
        }
        if (c == '"') { v.t = Json::Str; v.s = str(); return v; }
        if (lit("true")) { v.t = Json::Bool; v.b = true; return v; }
        if (lit("false")) { v.t = Json::Bool; return v; }
        if (lit("null")) return v;
        if (c == '-' || (c >= '0' && c <= '9')) {
            const char* s = p_;
            if (*p_ == '-') ++p_;
            while (p_ < e_ && ((*p_ >= '0' && *p_ <= '9') || *p_ == '.' || *p_ == 'e' || *p_ == 'E' || *p_ == '+' || *p_ == '-')) ++p_;
            v.t = Json::Num;
            v.n = std::strtod(std::string(s, p_).c_str(), nullptr);
            return v;
        }
        fail(std::string("unexpected '") + c + "'");
    }
    static void utf8(std::string& out, uint32_t cp) {
        if (cp < 0x80) out.push_back((char)cp);
        else if (cp < 0x800) { out.push_back((char)(0xC0 | (cp >> 6))); out.push_back((char)(0x80 | (cp & 0x3F))); }
        else if (cp < 0x10000) {
            out.push_back((char)(0xE0 | (cp >> 12)));
            out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            out.push_back((char)(0x80 | (cp & 0x3F)));
        } else {
            out.push_back((char)(0xF0 | (cp >> 18)));
            out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
            out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            out.push_back((char)(0x80 | (cp & 0x3F)));
        }
    }
    uint32_t hex4() {
        if (e_ - p_ < 4) fail("short \\u escape");
        uint32_t v = 0;
        for (int k = 0; k < 4; ++k) {
            const char h = *p_++;
            v <<= 4;
            if (h >= '0' && h <= '9') v |= (uint32_t)(h - '0');
            else if (h >= 'a' && h <= 'f') v |= (uint32_t)(h - 'a' + 10);
            else if (h >= 'A' && h <= 'F') v |= (uint32_t)(h - 'A' + 10);
            else fail("bad \\u escape");
        }
        return v;
    }
    std::string str() {
        ++p_;   // opening quote
        std::string out;
        for (;;) {
            if (p_ >= e_) fail("unterminated string");
            const char c = *p_++;
            if (c == '"') return out;
            if ((unsigned char)c < 0x20) fail("control character in string");
            if (c != '\\') { out.push_back(c); continue; }
            if (p_ >= e_) fail("unterminated escape");
            const char x = *p_++;
            switch (x) {
                case '"': out.push_back('"'); break;
                case '\\': out.push_back('\\'); break;
                case '/': out.push_back('/'); break;
                case 'b': out.push_back('\b'); break;
                case 'f': out.push_back('\f'); break;
                case 'n': out.push_back('\n'); break;
                case 'r': out.push_back('\r'); break;
                case 't': out.push_back('\t'); break;
                case 'u': {
                    uint32_t cp = hex4();
                    if (cp >= 0xD800 && cp < 0xDC00) {   // surrogate pair
                        if (e_ - p_ < 6 || p_[0] != '\\' || p_[1] != 'u') fail("lone surrogate");
                        p_ += 2;
                        const uint32_t lo = hex4();
                        if (lo < 0xDC00 || lo >= 0xE000) fail("bad surrogate pair");
                        cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                    }
                    utf8(out, cp);
                    break;
                }
                default: fail(std::string("bad escape \\") + x);
            }
        }
    }
};

std::string slurp(const std::string& path, const char* what) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw DataError(std::string("Cannot open ") + what + ": " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

// ---------------------------------------------------------------------------------------------
// images
// ---------------------------------------------------------------------------------------------
struct Image {
    int h = 0, w = 0, c = 0, bits = 8;   // c: 1 gray, 2 gray+alpha, 3 rgb, 4 rgba; bits 8 or 16
    std::vector<uint16_t> px;            // h*w*c samples, host order
};

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

Image decode_png(const std::string& bytes, const std::string& path) {
    const uint8_t* d = reinterpret_cast<const uint8_t*>(bytes.data());
    const size_t n = bytes.size();
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
    if (n < 8 || std::memcmp(d, sig, 8) != 0) throw DataError("not a PNG file: " + path);
    int w = 0, h = 0, bits = 0, ctype = -1, interlace = 0;
    std::vector<uint8_t> idat, plte;
    size_t p = 8;
    bool end = false;
    while (p + 12 <= n && !end) {
        const uint32_t len = be32(d + p);
        if (p + 12 + (size_t)len > n) throw DataError("truncated PNG chunk in " + path);
        const std::string type(reinterpret_cast<const char*>(d + p + 4), 4);
        const uint8_t* c = d + p + 8;
        if (type == "IHDR") {
            if (len < 13) throw DataError("bad IHDR in " + path);
            w = (int)be32(c); h = (int)be32(c + 4); bits = c[8]; ctype = c[9]; interlace = c[12];
        } else if (type == "PLTE") {
            plte.assign(c, c + len);
        } else if (type == "IDAT") {
            idat.insert(idat.end(), c, c + len);
        } else if (type == "IEND") {
            end = true;
        }
        p += 12 + len;
    }
    if (w <= 0 || h <= 0 || w > (1 << 16) || h > (1 << 16)) throw DataError("bad PNG dimensions in " + path);
    if (interlace) throw DataError("interlaced PNG is not supported: " + path);
    int ch;
    switch (ctype) {
        case 0: ch = 1; break;
        case 2: ch = 3; break;
        case 3: ch = 1; break;
        case 4: ch = 2; break;
        case 6: ch = 4; break;
        default: throw DataError("bad PNG colour type in " + path);
    }
    if (!((bits == 8 || bits == 16) && (ctype != 3 || bits == 8)))
        throw DataError("PNG bit depth " + std::to_string(bits) + " (colour type " + std::to_string(ctype) +
                        ") is not supported: " + path);
    const int bpp = ch * bits / 8;   // bytes per pixel (the filters' left neighbour distance)
    const size_t stride = (size_t)w * bpp;
    std::vector<uint8_t> raw((stride + 1) * (size_t)h);
    uLongf rawlen = (uLongf)raw.size();
    if (uncompress(raw.data(), &rawlen, idat.data(), (uLong)idat.size()) != Z_OK || rawlen != raw.size())
        throw DataError("corrupt PNG image data in " + path);
    std::vector<uint8_t> img(stride * (size_t)h);
    for (int y = 0; y < h; ++y) {
        const uint8_t ft = raw[(size_t)y * (stride + 1)];
        const uint8_t* in = raw.data() + (size_t)y * (stride + 1) + 1;
        uint8_t* out = img.data() + (size_t)y * stride;
        const uint8_t* up = y ? out - stride : nullptr;
        for (size_t i = 0; i < stride; ++i) {
            const int a = i >= (size_t)bpp ? out[i - bpp] : 0;
            const int b = up ? up[i] : 0;
            const int cc = (up && i >= (size_t)bpp) ? up[i - bpp] : 0;
            int v;
            switch (ft) {
                case 0: v = in[i]; break;
                case 1: v = in[i] + a; break;
                case 2: v = in[i] + b; break;
                case 3: v = in[i] + ((a + b) >> 1); break;
                case 4: {
                    const int pp = a + b - cc, pa = std::abs(pp - a), pb = std::abs(pp - b), pc = std::abs(pp - cc);
                    v = in[i] + ((pa <= pb && pa <= pc) ? a : pb <= pc ? b : cc);
                    break;
                }
                default: throw DataError("bad PNG filter type in " + path);
            }
            out[i] = (uint8_t)v;
        }
    }
    Image im;
    im.h = h; im.w = w; im.bits = bits;
    if (ctype == 3) {   // palette -> RGB
        im.c = 3;
        im.px.resize((size_t)h * w * 3);
        for (size_t i = 0; i < (size_t)h * w; ++i) {
            const size_t k = (size_t)img[i] * 3;
            if (k + 2 >= plte.size()) throw DataError("PNG palette index out of range in " + path);
            for (int q = 0; q < 3; ++q) im.px[i * 3 + q] = plte[k + q];
        }
        return im;
    }
    im.c = ch;
    im.px.resize((size_t)h * w * ch);
    if (bits == 8) {
        for (size_t i = 0; i < im.px.size(); ++i) im.px[i] = img[i];
    } else {
        for (size_t i = 0; i < im.px.size(); ++i) im.px[i] = (uint16_t)(img[2 * i] << 8 | img[2 * i + 1]);   // big-endian
    }
    return im;
}

Image decode_pnm(const std::string& bytes, const std::string& path) {
    // P5 (gray) / P6 (rgb), maxval <= 65535 (two big-endian bytes per sample above 255)
    size_t p = 0;
    auto token = [&]() {
        for (;;) {
            while (p < bytes.size() && std::isspace((unsigned char)bytes[p])) ++p;
            if (p < bytes.size() && bytes[p] == '#') {
                while (p < bytes.size() && bytes[p] != '\n') ++p;
                continue;
            }
            break;
        }
        const size_t s = p;
        while (p < bytes.size() && !std::isspace((unsigned char)bytes[p])) ++p;
        return bytes.substr(s, p - s);
    };
    const std::string magic = token();
    if (magic != "P5" && magic != "P6") throw DataError("not a binary PGM/PPM file: " + path);
    const int w = std::atoi(token().c_str()), h = std::atoi(token().c_str()), maxv = std::atoi(token().c_str());
    ++p;   // the single whitespace before the raster
    if (w <= 0 || h <= 0 || maxv <= 0 || maxv > 65535) throw DataError("bad PNM header in " + path);
    Image im;
    im.h = h; im.w = w; im.c = magic == "P6" ? 3 : 1; im.bits = maxv > 255 ? 16 : 8;
    const size_t count = (size_t)h * w * im.c, bps = maxv > 255 ? 2 : 1;
    if (p + count * bps > bytes.size()) throw DataError("truncated PNM raster in " + path);
    im.px.resize(count);
    const uint8_t* r = reinterpret_cast<const uint8_t*>(bytes.data()) + p;
    for (size_t i = 0; i < count; ++i) im.px[i] = bps == 2 ? (uint16_t)(r[2 * i] << 8 | r[2 * i + 1]) : r[i];
    return im;
}

std::string lower_ext(const fs::path& p) {
    std::string e = p.extension().string();
    std::transform(e.begin(), e.end(), e.begin(), [](unsigned char c) { return (char)std::tolower(c); });
    return e;
}

Image decode_jpeg(const std::string& bytes, const std::string& path) {
    cad::jpeg::Decoded d;
    try {
        d = cad::jpeg::decode(reinterpret_cast<const uint8_t*>(bytes.data()), bytes.size());
    } catch (const std::exception& e) {
        throw DataError(std::string(e.what()) + ": " + path);
    }
    Image im;
    im.h = d.h;
    im.w = d.w;
    im.c = d.c;
    im.px.assign(d.px.begin(), d.px.end());
    return im;
}

Image decode_image(const std::string& path) {
    const std::string ext = lower_ext(path);
    const std::string bytes = slurp(path, "image");
    if (ext == ".jpg" || ext == ".jpeg") return decode_jpeg(bytes, path);
    if (ext == ".png") return decode_png(bytes, path);
    if (ext == ".ppm" || ext == ".pgm" || ext == ".pnm") return decode_pnm(bytes, path);
    throw DataError("unsupported image format: " + path);
}

// loadRGB: imread(IMREAD_COLOR) (gray replicated, alpha dropped, 16-bit -> high byte) + BGR2RGB
void to_rgb8(const Image& im, uint8_t* out) {
    const size_t np = (size_t)im.h * im.w;
    for (size_t i = 0; i < np; ++i)
        for (int q = 0; q < 3; ++q) {
            const int src = im.c >= 3 ? q : 0;
            const uint16_t v = im.px[i * im.c + src];
            out[i * 3 + q] = (uint8_t)(im.bits == 16 ? v >> 8 : v);
        }
}

// loadDepth: imread(IMREAD_UNCHANGED): single channel only; 16-bit -> metres / 1000, 8-bit -> scale 1
float to_depth16(const Image& im, uint16_t* out, const std::string& path) {
    if (im.c != 1) throw DataError("depth map must be single-channel: " + path);
    std::copy(im.px.begin(), im.px.end(), out);
    return im.bits == 16 ? 1.0f / 1000.0f : 1.0f;
}

std::string first_file(const fs::path& dir, std::initializer_list<const char*> exts) {
    std::error_code ec;
    if (!fs::is_directory(dir, ec)) return "";
    std::vector<std::string> names;
    for (const auto& e : fs::directory_iterator(dir, ec)) {
        const std::string x = lower_ext(e.path());
        for (const char* want : exts)
            if (x == want) names.push_back(e.path().string());
    }
    std::sort(names.begin(), names.end());
    return names.empty() ? "" : names.front();
}

// synthetic decoded samples (data.dataset_name "synthetic" through the same ring): a smooth textured
// rgb and a u16 depth field with holes, deterministic per (seed, index)
uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

}  // namespace

struct cad_dataset {
    struct Item {
        std::string dir, sensor;
    };
    std::vector<Item> items;
    bool synthetic = false;
    int syn_h = 0, syn_w = 0;
    uint32_t seed = 0;
    int64_t n = 0;

    // one decoded sample: rgb HWC u8 (RGB), depth HW u16, info
    void read(int64_t i, std::vector<uint8_t>& rgb, std::vector<uint16_t>& depth, cad_decoded_info& info) const {
        if (i < 0 || i >= n) throw std::out_of_range("Sample index out of range");
        info = cad_decoded_info{};
        if (synthetic) {
            const int H = syn_h, W = syn_w;
            rgb.resize((size_t)H * W * 3);
            depth.resize((size_t)H * W);
            const double ph = 0.37 * (double)i;
            for (int y = 0; y < H; ++y)
                for (int x = 0; x < W; ++x) {
                    const uint64_t r = mix64(((uint64_t)seed << 40) ^ ((uint64_t)i << 24) ^ (uint64_t)(y * W + x));
                    const double u = (double)x / W, v = (double)y / H;
                    for (int q = 0; q < 3; ++q) {
                        const double t = 0.5 + 0.35 * std::sin(6.2832 * (u * (1.0 + q) + v * 0.7 + ph)) + 0.15 * ((r >> (8 * q) & 255) / 255.0 - 0.5);
                        rgb[((size_t)y * W + x) * 3 + q] = (uint8_t)std::min(255.0, std::max(0.0, t * 255.0));
                    }
                    const double dm = 0.5 + 9.0 * (0.5 + 0.5 * std::sin(6.2832 * (u * 1.3 + v * 0.7 + 0.1 * (double)i)));
                    const bool hole = (r >> 32 & 1023) < 154 || y < H / 16;
                    depth[(size_t)y * W + x] = hole ? 0 : (uint16_t)std::min(9500.0, std::max(500.0, dm * 1000.0));
                }
            info.h0 = info.dh0 = H;
            info.w0 = info.dw0 = W;
            info.depth_scale = 1.0f / 1000.0f;
            const bool even = i % 2 == 0;
            const float sx = (float)W / 640.f, sy = (float)H / 480.f;
            info.K[0] = (even ? 518.858f : 570.342f) * sx;
            info.K[2] = (even ? 325.582f : 320.0f) * sx;
            info.K[4] = (even ? 519.470f : 570.342f) * sy;
            info.K[5] = (even ? 253.736f : 240.0f) * sy;
            info.K[8] = 1.f;
            return;
        }
        const Item& it = items[(size_t)i];
        const std::string rgb_path = first_file(fs::path(it.dir) / "image", {".jpg", ".jpeg", ".png", ".ppm", ".pnm"});
        if (rgb_path.empty()) throw DataError("RGB image not found: " + it.dir);
        const std::string depth_path = first_file(fs::path(it.dir) / "depth", {".png", ".pgm", ".pnm"});
        if (depth_path.empty()) throw DataError("Depth image not found: " + it.dir);
        const Image ri = decode_image(rgb_path);
        rgb.resize((size_t)ri.h * ri.w * 3);
        to_rgb8(ri, rgb.data());
        const Image di = decode_image(depth_path);
        depth.resize((size_t)di.h * di.w);
        info.depth_scale = to_depth16(di, depth.data(), depth_path);
        info.h0 = ri.h; info.w0 = ri.w; info.dh0 = di.h; info.dw0 = di.w;
        // loadIntrinsics: 9 floats with operator>> (a short file leaves zeros, like the reference's vector)
        std::ifstream kf(fs::path(it.dir) / "intrinsics.txt");
        if (!kf) throw DataError("Cannot open intrinsics file: " + (fs::path(it.dir) / "intrinsics.txt").string());
        for (int k = 0; k < 9; ++k) kf >> info.K[k];
    }
};

// ---------------------------------------------------------------------------------------------
// prefetch ring
// ---------------------------------------------------------------------------------------------
namespace {

struct Pinned {
    void* p = nullptr;
    size_t cap = 0;
    void reserve(size_t n) {
        if (n <= cap) return;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        if (hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess) throw DataError("pinned host allocation failed");
        cap = n;
    }
    ~Pinned() {
        if (p) (void)hipHostFree(p);
    }
};
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

}  // namespace

struct cad_loader {
    struct Part {   // one sample of a slot
        Pinned rgb, depth;
        DevBuf drgb, ddepth;
        cad_decoded_info info{};
    };
    struct Slot {
        std::vector<Part> parts;
        int64_t batch = -1;   // batch index held (or being filled)
        int n = 0, pending = 0;
        bool ready = false, used = false;
        std::string err;
        hipEvent_t copied = nullptr, consumed = nullptr;
    };
    struct Task {
        int slot, part;
        int64_t sample, batch;
        bool wait_copy;   // the slot held an uploaded batch before: wait for that upload to finish
    };

    const cad_dataset* ds = nullptr;
    int B = 0, H = 0, W = 0, device = 0;
    bool aug = false;
    cad_aug_sampler* sampler = nullptr;
    cad_batcher* batcher = nullptr;
    hipStream_t copy = nullptr;
    std::vector<Slot> slots;
    std::vector<int64_t> order;
    int64_t nbatches = 0, issued = 0, consumed = 0;
    uint64_t epoch = 0;
    std::vector<std::thread> workers;
    std::mutex mu;
    std::condition_variable cv_work, cv_ready;
    std::deque<Task> tasks;
    int inflight = 0;   // tasks popped by a worker and not finished
    bool stop = false;
    std::vector<cad_sample> smp;

    // queue the decode of batch `b` into its slot (caller holds mu)
    void issue(int64_t b) {
        Slot& s = slots[(size_t)(b % (int64_t)slots.size())];
        const int64_t first = b * B;
        s.batch = b;
        s.n = (int)std::min<int64_t>(B, (int64_t)order.size() - first);
        s.pending = s.n;
        s.ready = false;
        s.err.clear();
        for (int j = 0; j < s.n; ++j)
            tasks.push_back({(int)(b % (int64_t)slots.size()), j, order[(size_t)(first + j)], b, s.used});
        cv_work.notify_all();
    }

    void worker() {
        (void)hipSetDevice(device);
        std::vector<uint8_t> rgb;
        std::vector<uint16_t> dep;
        for (;;) {
            Task t;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv_work.wait(lk, [&] { return stop || !tasks.empty(); });
                if (stop) return;
                t = tasks.front();
                tasks.pop_front();
                ++inflight;
            }
            Slot& s = slots[(size_t)t.slot];
            std::string err;
            try {
                // the previous occupant's upload must have left the pinned buffers
                if (t.wait_copy && hipEventSynchronize(s.copied) != hipSuccess) throw DataError("upload failed");
                cad_decoded_info info;
                ds->read(t.sample, rgb, dep, info);
                Part& p = s.parts[(size_t)t.part];
                p.rgb.reserve(rgb.size());
                p.depth.reserve(dep.size() * 2);
                std::memcpy(p.rgb.p, rgb.data(), rgb.size());
                std::memcpy(p.depth.p, dep.data(), dep.size() * 2);
                p.info = info;
            } catch (const std::exception& e) {
                err = "sample " + std::to_string(t.sample) + ": " + e.what();
            }
            std::lock_guard<std::mutex> lk(mu);
            --inflight;
            if (s.batch == t.batch) {   // (else stale: the epoch was restarted)
                if (!err.empty() && s.err.empty()) s.err = err;
                if (--s.pending == 0) s.ready = true;
            }
            cv_ready.notify_all();
        }
    }

    void drain() {
        // drop queued decodes and wait for the ones a worker already holds
        std::unique_lock<std::mutex> lk(mu);
        tasks.clear();
        for (auto& s : slots) s.batch = -1;
        cv_ready.wait(lk, [&] { return inflight == 0; });
    }
};

extern "C" {

cad_status cad_dataset_open(const char* manifest_path, const char* const* sensors, int n_sensors, cad_dataset** out) {
    return data_guard([&] {
        if (!manifest_path || !out || n_sensors < 0 || (n_sensors > 0 && !sensors)) throw DataError("bad arguments");
        const Json m = JsonParser(slurp(manifest_path, "manifest file"), manifest_path).parse();
        std::vector<std::string> allowed = {"kv1", "kv2", "realsense", "xtion"};   // constructor default :25
        if (n_sensors > 0) allowed.assign(sensors, sensors + n_sensors);
        const Json* images = m.get("images");
        if (!images || images->t != Json::Arr) throw DataError(std::string(manifest_path) + ": no \"images\" array");
        auto ds = std::make_unique<cad_dataset>();
        for (const Json& im : images->a) {
            const Json* valid = im.get("valid");
            if (!valid || valid->t != Json::Bool || !valid->b) continue;
            const Json* sensor = im.get("sensor_type");
            const Json* path = im.get("path");
            if (!sensor || sensor->t != Json::Str || !path || path->t != Json::Str)
                throw DataError(std::string(manifest_path) + ": image entry without sensor_type/path");
            if (std::find(allowed.begin(), allowed.end(), sensor->s) == allowed.end()) continue;
            std::error_code ec;
            if (!fs::exists(fs::path(path->s) / "intrinsics.txt", ec)) continue;
            ds->items.push_back({path->s, sensor->s});
        }
        ds->n = (int64_t)ds->items.size();
        *out = ds.release();
    });
}

cad_status cad_jpeg_decode(const uint8_t* data, int64_t size, uint8_t* out, int64_t cap, int* height, int* width,
                           int* channels) {
    return data_guard([&] {
        if (!data || size < 0) throw DataError("bad arguments");
        const cad::jpeg::Decoded d = cad::jpeg::decode(data, (size_t)size);
        if (height) *height = d.h;
        if (width) *width = d.w;
        if (channels) *channels = d.c;
        if (out) {
            if (cap < (int64_t)d.px.size()) throw DataError("output buffer too small");
            std::memcpy(out, d.px.data(), d.px.size());
        }
    });
}

cad_status cad_dataset_synthetic(int64_t n, int height, int width, uint32_t seed, cad_dataset** out) {
    return data_guard([&] {
        if (!out || n < 0 || height < 1 || width < 1) throw DataError("bad arguments");
        auto ds = std::make_unique<cad_dataset>();
        ds->synthetic = true;
        ds->n = n;
        ds->syn_h = height;
        ds->syn_w = width;
        ds->seed = seed;
        *out = ds.release();
    });
}

void cad_dataset_destroy(cad_dataset* d) { delete d; }
int64_t cad_dataset_size(const cad_dataset* d) { return d ? d->n : -1; }

const char* cad_dataset_image_dir(const cad_dataset* d, int64_t i) {
    if (!d || d->synthetic || i < 0 || i >= d->n) return nullptr;
    return d->items[(size_t)i].dir.c_str();
}

cad_status cad_dataset_read(const cad_dataset* d, int64_t i, uint8_t* rgb, int64_t rgb_cap, uint16_t* depth,
                            int64_t depth_cap, cad_decoded_info* info) {
    return data_guard([&] {
        if (!d || !info) throw DataError("bad arguments");
        std::vector<uint8_t> r;
        std::vector<uint16_t> dd;
        d->read(i, r, dd, *info);
        if (rgb) {
            if (rgb_cap < (int64_t)r.size()) throw DataError("rgb buffer too small");
            std::memcpy(rgb, r.data(), r.size());
        }
        if (depth) {
            if (depth_cap < (int64_t)dd.size()) throw DataError("depth buffer too small");
            std::memcpy(depth, dd.data(), dd.size() * 2);
        }
    });
}

cad_status cad_loader_create(const cad_dataset* ds, int batch, int height, int width, const cad_aug_config* aug,
                             uint32_t seed, int threads, int slots, int device, cad_loader** out) {
    return data_guard([&] {
        if (!ds || !out || batch < 1 || height < 1 || width < 1 || threads < 1 || slots < 2)
            throw DataError("bad loader arguments");
        auto L = std::make_unique<cad_loader>();
        L->ds = ds;
        L->B = batch; L->H = height; L->W = width; L->device = device;
        if (hipSetDevice(device) != hipSuccess) throw DataError("bad device");
        if (cad_batcher_create(batch, height, width, device, &L->batcher) != CAD_OK) throw DataError(cad_last_error());
        if (aug) {
            L->aug = true;
            if (cad_aug_sampler_create(aug, seed, &L->sampler) != CAD_OK) throw DataError(cad_last_error());
        }
        if (hipStreamCreateWithFlags(&L->copy, hipStreamNonBlocking) != hipSuccess) throw DataError("stream creation failed");
        L->slots.resize((size_t)slots);
        for (auto& s : L->slots) {
            s.parts.resize((size_t)batch);
            if (hipEventCreateWithFlags(&s.copied, hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&s.consumed, hipEventDisableTiming) != hipSuccess)
                throw DataError("event creation failed");
        }
        L->smp.resize((size_t)batch);
        for (int t = 0; t < threads; ++t) L->workers.emplace_back([p = L.get()] { p->worker(); });
        *out = L.release();
    });
}

void cad_loader_destroy(cad_loader* L) {
    if (!L) return;
    {
        std::lock_guard<std::mutex> lk(L->mu);
        L->stop = true;
        L->tasks.clear();
    }
    L->cv_work.notify_all();
    for (auto& t : L->workers) t.join();
    (void)hipSetDevice(L->device);
    if (L->copy) (void)hipStreamSynchronize(L->copy);
    for (auto& s : L->slots) {
        if (s.consumed) (void)hipEventSynchronize(s.consumed);
        if (s.copied) (void)hipEventDestroy(s.copied);
        if (s.consumed) (void)hipEventDestroy(s.consumed);
    }
    if (L->copy) (void)hipStreamDestroy(L->copy);
    if (L->sampler) cad_aug_sampler_destroy(L->sampler);
    if (L->batcher) cad_batcher_destroy(L->batcher);
    delete L;
}

cad_status cad_loader_start_epoch(cad_loader* L, const int64_t* order, int64_t n) {
    return data_guard([&] {
        if (!L || n < 0 || (n > 0 && !order && n > L->ds->n)) throw DataError("bad arguments");
        L->drain();
        std::lock_guard<std::mutex> lk(L->mu);
        L->order.resize((size_t)n);
        for (int64_t k = 0; k < n; ++k) {
            const int64_t v = order ? order[k] : k;
            if (v < 0 || v >= L->ds->n) throw DataError("sample index out of range in the epoch order");
            L->order[(size_t)k] = v;
        }
        L->nbatches = (n + L->B - 1) / L->B;   // trainEpoch keeps the last partial batch (:262, :269-270)
        L->issued = L->consumed = 0;
        for (auto& s : L->slots) { s.batch = -1; s.ready = false; s.pending = 0; }
        while (L->issued < L->nbatches && L->issued < (int64_t)L->slots.size()) L->issue(L->issued++);
    });
}

int cad_loader_next(cad_loader* L, float* rgb, float* depth, float* K, void* stream) {
    int n = -1;
    const cad_status st = data_guard([&] {
        if (!L || !rgb || !depth || !K) throw DataError("bad arguments");
        if (L->consumed >= L->nbatches) { n = 0; return; }
        const int64_t b = L->consumed;
        cad_loader::Slot& s = L->slots[(size_t)(b % (int64_t)L->slots.size())];
        {
            std::unique_lock<std::mutex> lk(L->mu);
            L->cv_ready.wait(lk, [&] { return s.batch == b && s.ready; });
            if (!s.err.empty()) throw DataError(s.err);
        }
        hipStream_t cs = reinterpret_cast<hipStream_t>(stream);
        if (hipSetDevice(L->device) != hipSuccess) throw DataError("bad device");
        // the slot's device buffers are free once the previous batch in it has been assembled
        if (s.used && hipStreamWaitEvent(L->copy, s.consumed, 0) != hipSuccess) throw DataError("stream wait failed");
        for (int j = 0; j < s.n; ++j) {
            cad_loader::Part& p = s.parts[(size_t)j];
            const size_t nr = (size_t)p.info.h0 * p.info.w0 * 3, nd = (size_t)p.info.dh0 * p.info.dw0 * 2;
            for (const auto& bufn : {std::make_pair(&p.drgb, nr), std::make_pair(&p.ddepth, nd)}) {
                DevBuf& db = *bufn.first;
                if (db.cap >= bufn.second) continue;
                if (s.used) (void)hipEventSynchronize(s.consumed);
                if (db.p) (void)hipFree(db.p);
                db.p = nullptr;
                if (hipMalloc(&db.p, bufn.second) != hipSuccess) throw DataError("device allocation failed");
                db.cap = bufn.second;
            }
            if (hipMemcpyAsync(p.drgb.p, p.rgb.p, nr, hipMemcpyHostToDevice, L->copy) != hipSuccess ||
                hipMemcpyAsync(p.ddepth.p, p.depth.p, nd, hipMemcpyHostToDevice, L->copy) != hipSuccess)
                throw DataError("upload failed");
            cad_sample& c = L->smp[(size_t)j];
            c = cad_sample{};
            c.rgb = static_cast<const uint8_t*>(p.drgb.p);
            c.depth = static_cast<const uint16_t*>(p.ddepth.p);
            c.h0 = p.info.h0; c.w0 = p.info.w0; c.dh0 = p.info.dh0; c.dw0 = p.info.dw0;
            c.bgr = 0;
            c.depth_scale = p.info.depth_scale;
            std::memcpy(c.K, p.info.K, sizeof c.K);
            // augmentSample's draws, in sample order on this thread (the loader's single rng_)
            if (L->sampler && cad_aug_sampler_draw(L->sampler, L->H, L->W, &c) != CAD_OK) throw DataError(cad_last_error());
        }
        if (hipEventRecord(s.copied, L->copy) != hipSuccess || hipStreamWaitEvent(cs, s.copied, 0) != hipSuccess)
            throw DataError("event failed");
        if (cad_batcher_assemble(L->batcher, L->smp.data(), s.n, rgb, depth, K, stream) != CAD_OK)
            throw DataError(cad_last_error());
        if (hipEventRecord(s.consumed, cs) != hipSuccess) throw DataError("event failed");
        n = s.n;
        std::lock_guard<std::mutex> lk(L->mu);
        s.used = true;
        s.ready = false;
        ++L->consumed;
        if (L->issued < L->nbatches) L->issue(L->issued++);   // refill this slot (the worker waits for `copied`)
    });
    return st == CAD_OK ? n : -1;
}

}  // extern "C"

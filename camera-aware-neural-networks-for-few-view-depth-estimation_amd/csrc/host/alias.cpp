// Launch-level aliasing guard (kernels.hpp CAD_NO_ALIAS).  A kernel that reads a buffer while another
// workgroup of the same launch writes it races (round 5: a window dgrad split-stored its bf16 up half
// into dYs while reading dYs as its dZ; every B = 2 test passed, the bs32 one did not).  With
// CAD_ALIAS_CHECK=1 every instrumented launcher compares the byte ranges of its outputs with those of
// its inputs before launching and refuses an overlap: std::invalid_argument naming both operands,
// which the C ABI returns as CAD_ERR_INVALID (cad_last_error).  CAD_ALIAS_CHECK=log:<path> appends the
// finding to <path> and launches anyway.  Unset / 0: the launchers test one cached int.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <sstream>
#include <stdexcept>
#include <string>

#include "../kernels/kernels.hpp"

namespace cad {

namespace {
std::string g_log_path;

int read_mode() {
    const char* e = std::getenv("CAD_ALIAS_CHECK");
    if (!e || !e[0] || (e[0] == '0' && !e[1])) return 0;
    if (std::strncmp(e, "log:", 4) == 0) {
        g_log_path = e + 4;
        return 2;
    }
    return 1;
}

// byte range [lo, hi) a view touches, and its row pitch / row width in bytes
struct Span {
    uintptr_t lo = 0, hi = 0;
    int64_t pitch = 0, width = 0;
};
Span span_of(const AliasView& v) {
    Span s;
    const uintptr_t base = reinterpret_cast<uintptr_t>(v.p);
    s.lo = base + (uintptr_t)(v.coff * v.es);
    s.hi = base + (uintptr_t)(((v.rows - 1) * v.ld + v.coff + v.cols) * v.es);
    s.pitch = v.ld * v.es;
    s.width = v.cols * v.es;
    return s;
}
bool empty(const AliasView& v) { return !v.p || v.rows <= 0 || v.cols <= 0; }

std::string describe(const AliasView& v) {
    std::ostringstream o;
    o << v.what << " (" << (v.es == 2 ? "bf16" : v.es == 1 ? "u8" : v.es == 8 ? "f64" : "fp32") << " rows " << v.rows
      << " x cols " << v.cols << ", ld " << v.ld << ", coff " << v.coff << ", at " << v.p << ")";
    return o.str();
}
}  // namespace

int g_alias_mode = -1;   // -1: CAD_ALIAS_CHECK not read yet (cad_set_alias_check sets it)

int alias_mode() {
    if (g_alias_mode < 0) g_alias_mode = read_mode();
    return g_alias_mode;
}

bool views_overlap(const AliasView& a, const AliasView& b) {
    if (empty(a) || empty(b)) return false;
    const Span x = span_of(a), y = span_of(b);
    if (x.hi <= y.lo || y.hi <= x.lo) return false;
    // two row views with the same pitch touch disjoint bytes when their column ranges never meet
    // modulo the pitch (the skip / up halves of a concat buffer)
    if (x.pitch == y.pitch && x.pitch > 0 && x.width <= x.pitch && y.width <= y.pitch && a.rows > 1 && b.rows > 1) {
        int64_t d = (int64_t)(y.lo - x.lo) % x.pitch;
        if (d < 0) d += x.pitch;
        return d < x.width || d + y.width > x.pitch;
    }
    return true;
}

void alias_check_impl(const char* op, std::initializer_list<AliasView> outs, std::initializer_list<AliasView> ins,
                      bool same_view_ok) {
    for (const AliasView& o : outs)
        for (const AliasView& i : ins) {
            // an elementwise pass may run in place: each thread reads an element, then writes that element
            if (same_view_ok && o.p == i.p && o.ld == i.ld && o.coff == i.coff && o.cols == i.cols && o.es == i.es &&
                o.rows == i.rows)
                continue;
            if (!views_overlap(o, i)) continue;
            const std::string msg = std::string("alias: ") + op + " writes " + describe(o) + " over its input " +
                                    describe(i) + " (a launch may not read what it writes unless it is declared in place)";
            if (alias_mode() == 2) {
                static std::mutex mu;
                std::lock_guard<std::mutex> lk(mu);
                if (FILE* f = std::fopen(g_log_path.c_str(), "a")) {
                    std::fprintf(f, "%s\n", msg.c_str());
                    std::fclose(f);
                }
                continue;
            }
            throw std::invalid_argument(msg);
        }
}

}  // namespace cad

// C ABI (cad.h): the guard's switch and its overlap rule, for the tests
extern "C" {
int cad_set_alias_check(int mode) {
    const int prev = cad::alias_mode();
    // (log mode needs the path CAD_ALIAS_CHECK=log:<path> named: it can be restored, not chosen)
    cad::g_alias_mode = mode == 1 ? 1 : (mode == 2 && !cad::g_log_path.empty()) ? 2 : 0;
    return prev;
}
int cad_alias_views_overlap(const void* a, int64_t arows, int64_t ald, int64_t acoff, int64_t acols, int aes,
                            const void* b, int64_t brows, int64_t bld, int64_t bcoff, int64_t bcols, int bes) {
    return cad::views_overlap(cad::aview(a, arows, ald, acoff, acols, aes, "a"),
                              cad::aview(b, brows, bld, bcoff, bcols, bes, "b")) ? 1 : 0;
}
}

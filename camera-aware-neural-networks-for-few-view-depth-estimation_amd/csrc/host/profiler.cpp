// In-library launch profiler: when enabled, every MFMA GEMM launch is bracketed by a pair of
// hipEvents recorded on the SAME stream the kernel is launched on, tagged with the kernel symbol
// (as rocprofv3 prints it) and its algorithmic FLOPs (2*M*N*K).  bench.py reads the aggregate to
// report roofline.achieved for the dominant kernel; rocprofv3 --kernel-trace --stats of the same
// command cross-checks the average durations.  Disabled: one predictable branch per launch.
// cad_profile_only(name): events only around the launches of that kernel (the others are not timed):
// two event records per launch cost ~5 us of stream time each, so a timed region that brackets every
// GEMM runs ~1-2 % slower than one that brackets only the kernel whose roofline is reported.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../../include/cad/cad.h"
#include "../kernels/kernels.hpp"

namespace cad {
namespace {
struct Rec {
    int name_id;
    double flops;
    hipEvent_t a, b;
};
struct ProfState {
    bool on = false;
    std::vector<std::string> names;
    std::map<std::string, int> ids;
    std::vector<Rec> recs;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pool;
    size_t used = 0;
    std::string only;    // non-empty: time only launches of this kernel
    bool skipped = false;   // the last push was filtered out (its pop records nothing)
};
ProfState& ps() {
    static ProfState s;
    return s;
}
}  // namespace

bool prof_enabled() { return ps().on; }

void prof_push(const char* name, double flops, hipStream_t st) {
    ProfState& s = ps();
    s.skipped = !s.only.empty() && std::strcmp(name, s.only.c_str()) != 0;
    if (s.skipped) return;
    auto it = s.ids.find(name);
    int id;
    if (it == s.ids.end()) {
        id = (int)s.names.size();
        s.names.push_back(name);
        s.ids[name] = id;
    } else {
        id = it->second;
    }
    if (s.used == s.pool.size()) {
        hipEvent_t a, b;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
        s.pool.push_back({a, b});
    }
    auto ev = s.pool[s.used++];
    (void)hipEventRecord(ev.first, st);
    s.recs.push_back({id, flops, ev.first, ev.second});
}

void prof_pop(hipStream_t st) {
    ProfState& s = ps();
    if (s.skipped) {
        s.skipped = false;
        return;
    }
    (void)hipEventRecord(s.recs.back().b, st);
}

}  // namespace cad

extern "C" {

cad_status cad_profile_enable(int on) {
    cad::ps().on = on != 0;
    return CAD_OK;
}

cad_status cad_profile_only(const char* kernel_name) {
    cad::ps().only = kernel_name ? kernel_name : "";
    cad::ps().skipped = false;
    return CAD_OK;
}

cad_status cad_profile_reset(void) {
    cad::ps().recs.clear();
    cad::ps().used = 0;
    return CAD_OK;
}

// JSON: [{"name": ..., "launches": n, "ms": total, "gflop": total}, ...]; synchronises the events
int cad_profile_report(char* buf, int cap) {
    auto& s = cad::ps();
    std::vector<double> ms(s.names.size(), 0.0), gf(s.names.size(), 0.0);
    std::vector<int> n(s.names.size(), 0);
    for (auto& r : s.recs) {
        (void)hipEventSynchronize(r.b);
        float t = 0.f;
        (void)hipEventElapsedTime(&t, r.a, r.b);
        ms[r.name_id] += t;
        gf[r.name_id] += r.flops * 1e-9;
        n[r.name_id] += 1;
    }
    std::string out = "[";
    for (size_t i = 0; i < s.names.size(); ++i) {
        if (!n[i]) continue;
        char tmp[512];
        snprintf(tmp, sizeof(tmp), "%s{\"name\": \"%s\", \"launches\": %d, \"ms\": %.6f, \"gflop\": %.6f}",
                 out.size() > 1 ? ", " : "", s.names[i].c_str(), n[i], ms[i], gf[i]);
        out += tmp;
    }
    out += "]";
    if (buf && cap > 0) {
        snprintf(buf, (size_t)cap, "%s", out.c_str());
    }
    return (int)out.size() + 1;
}

}  // extern "C"

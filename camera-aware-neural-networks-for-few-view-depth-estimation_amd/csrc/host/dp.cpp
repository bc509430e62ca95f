// Data-parallel gradient exchange of the training step over RCCL (xGMI between the GPUs of a node).
//
// New relative to the reference, which is single-process and single-device (SURVEY.md §2
// "Parallelism strategies: none", §8(e)): one process per GPU, each with a full replica; the one
// exchange per step is the SUM all-reduce of the flat gradient slab, bucketed decoder-first and
// issued on a communication stream while the rest of the backward still runs (the backward stages
// finish in decreasing slab-offset order: head, dec1..dec4, bottleneck, enc4..enc1).  The 1/world
// mean is folded into clip_grad_norm_'s prescale, so clip and Adam stay one pass each and every
// replica applies the identical update.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../../include/cad/cad.h"

namespace cad {
void set_last_error(const std::string& msg);   // cad_api.cpp: the thread-local cad_last_error() text
}

// timing events of one backward_allreduce call (cad_comm_set_timing)
struct CommTimes {
    hipEvent_t bwd_end = nullptr;    // compute stream: after the last backward stage
    hipEvent_t released = nullptr;   // compute stream: after its wait for the last all-reduce
    hipEvent_t ar_start = nullptr;   // comm stream: the first bucket may start
    hipEvent_t ar_end = nullptr;     // comm stream: after the last all-reduce
};
constexpr int kMaxTimedCalls = 256;

struct cad_comm {
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0, device = 0;
    hipStream_t stream = nullptr;            // communication stream
    std::vector<hipEvent_t> ready;           // one per bucket slot: its stages are enqueued
    hipEvent_t done = nullptr;               // every issued all-reduce has completed
    // exchange accounting (cad_comm_stats_read)
    bool timing = false;
    std::vector<CommTimes> times;            // event sets, reused after each read
    int ntimed = 0;                          // sets recorded since the last read
    cad_comm_stats acc{};
};

namespace {

struct DpError : std::runtime_error {
    cad_status st;
    DpError(cad_status s, const std::string& m) : std::runtime_error(m), st(s) {}
};

#define DP_HIP(expr)                                                                                \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess) throw DpError(CAD_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)
#define DP_NCCL(expr)                                                                               \
    do {                                                                                            \
        ncclResult_t r_ = (expr);                                                                   \
        if (r_ != ncclSuccess) throw DpError(CAD_ERR_HIP, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

template <class F>
cad_status dp_guard(F&& f) {
    try {
        f();
        return CAD_OK;
    } catch (const DpError& e) {
        cad::set_last_error(e.what());
        return e.st;
    } catch (const std::exception& e) {
        cad::set_last_error(e.what());
        return CAD_ERR_INVALID;
    }
}

inline hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace

namespace {
// The overlapped exchange for any model with a staged backward (stage s writes only the gradients in
// its slab range; ranges decrease with s): every stage is enqueued on `stream`; when the stages of a
// bucket are enqueued, an event on `stream` gates the bucket's SUM all-reduce on the communicator's
// stream, so RCCL runs while the later stages do; `stream` finally waits for every all-reduce.
template <class Range, class Stage>
void staged_backward_allreduce(cad_comm* c, float* g, int ns, Range range, Stage stage, int64_t bucket_elems,
                               void* stream) {
    DP_HIP(hipSetDevice(c->device));
    std::vector<int64_t> off((size_t)ns), cnt((size_t)ns), boff((size_t)ns), bcnt((size_t)ns);
    std::vector<int> blast((size_t)ns);
    for (int s = 0; s < ns; ++s)
        if (range(s, &off[(size_t)s], &cnt[(size_t)s]) != CAD_OK) throw DpError(CAD_ERR_INVALID, "stage range");
    const int nb = cad_plan_grad_buckets(off.data(), cnt.data(), ns, std::max<int64_t>(bucket_elems, 1), boff.data(),
                                         bcnt.data(), blast.data());
    if (nb <= 0) throw DpError(CAD_ERR_INVALID, "no gradient buckets");
    while ((int)c->ready.size() < nb) {
        hipEvent_t e;
        DP_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        c->ready.push_back(e);
    }
    // timing events of this call (cad_comm_set_timing): a fresh set per call until the next read
    CommTimes* t = nullptr;
    if (c->timing && c->ntimed < kMaxTimedCalls) {
        if ((int)c->times.size() <= c->ntimed) {
            CommTimes n;
            for (hipEvent_t* e : {&n.bwd_end, &n.released, &n.ar_start, &n.ar_end}) DP_HIP(hipEventCreate(e));
            c->times.push_back(n);
        }
        t = &c->times[(size_t)c->ntimed];
    }
    int b = 0;
    for (int s = 0; s < ns; ++s) {
        const cad_status st = stage(s);
        if (st != CAD_OK) throw DpError(st, std::string("backward stage: ") + cad_last_error());
        if (b < nb && blast[(size_t)b] == s) {
            // the bucket's gradients are final once the work enqueued so far on `stream` is done
            DP_HIP(hipEventRecord(c->ready[(size_t)b], S(stream)));
            DP_HIP(hipStreamWaitEvent(c->stream, c->ready[(size_t)b], 0));
            if (t && b == 0) DP_HIP(hipEventRecord(t->ar_start, c->stream));
            DP_NCCL(ncclAllReduce(g + boff[(size_t)b], g + boff[(size_t)b], (size_t)bcnt[(size_t)b], ncclFloat32,
                                  ncclSum, c->comm, c->stream));
            c->acc.bytes += 4 * bcnt[(size_t)b];
            ++b;
        }
    }
    c->acc.buckets += nb;
    ++c->acc.calls;
    if (t) {
        DP_HIP(hipEventRecord(t->ar_end, c->stream));
        DP_HIP(hipEventRecord(t->bwd_end, S(stream)));
    }
    DP_HIP(hipEventRecord(c->done, c->stream));
    DP_HIP(hipStreamWaitEvent(S(stream), c->done, 0));   // clip / Adam see the reduced slab
    if (t) {
        DP_HIP(hipEventRecord(t->released, S(stream)));
        ++c->ntimed;
    }
}

}  // namespace

extern "C" {

int cad_plan_grad_buckets(const int64_t* stage_off, const int64_t* stage_cnt, int nstages, int64_t bucket_elems,
                          int64_t* bucket_off, int64_t* bucket_cnt, int* bucket_last_stage) {
    // greedy, in backward (stage) order: a bucket closes as soon as the union of its consecutive
    // stages' ranges holds >= bucket_elems floats, or at the last stage.  Consecutive stages are
    // adjacent slices of the slab (decreasing offsets), so a bucket is one contiguous range.
    if (!stage_off || !stage_cnt || nstages <= 0) return -1;
    int nb = 0;
    int64_t lo = -1, hi = -1;
    for (int s = 0; s < nstages; ++s) {
        if (stage_cnt[s] < 0) return -1;
        const int64_t a = stage_off[s], b = stage_off[s] + stage_cnt[s];
        lo = lo < 0 ? a : std::min(lo, a);
        hi = hi < 0 ? b : std::max(hi, b);
        if (hi - lo >= bucket_elems || s == nstages - 1) {
            if (bucket_off) bucket_off[nb] = lo;
            if (bucket_cnt) bucket_cnt[nb] = hi - lo;
            if (bucket_last_stage) bucket_last_stage[nb] = s;
            ++nb;
            lo = hi = -1;
        }
    }
    return nb;
}

cad_status cad_comm_get_unique_id(uint8_t id[CAD_COMM_ID_BYTES]) {
    return dp_guard([&] {
        if (!id) throw DpError(CAD_ERR_INVALID, "null id");
        static_assert(CAD_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");
        ncclUniqueId u;
        DP_NCCL(ncclGetUniqueId(&u));
        std::memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
    });
}

cad_status cad_comm_create(const uint8_t id[CAD_COMM_ID_BYTES], int nranks, int rank, int device, cad_comm** out) {
    return dp_guard([&] {
        if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks) throw DpError(CAD_ERR_INVALID, "bad communicator arguments");
        DP_HIP(hipSetDevice(device));
        auto c = new cad_comm();
        c->nranks = nranks; c->rank = rank; c->device = device;
        try {
            ncclUniqueId u;
            std::memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
            DP_NCCL(ncclCommInitRank(&c->comm, nranks, u, rank));
            DP_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
            DP_HIP(hipEventCreateWithFlags(&c->done, hipEventDisableTiming));
        } catch (...) {
            cad_comm_destroy(c);
            throw;
        }
        *out = c;
    });
}

void cad_comm_destroy(cad_comm* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    for (hipEvent_t e : c->ready) (void)hipEventDestroy(e);
    for (CommTimes& t : c->times)
        for (hipEvent_t e : {t.bwd_end, t.released, t.ar_start, t.ar_end})
            if (e) (void)hipEventDestroy(e);
    if (c->done) (void)hipEventDestroy(c->done);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int cad_comm_rank(const cad_comm* c) { return c ? c->rank : -1; }
int cad_comm_size(const cad_comm* c) { return c ? c->nranks : -1; }

cad_status cad_comm_set_timing(cad_comm* c, int enable) {
    return dp_guard([&] {
        if (!c) throw DpError(CAD_ERR_INVALID, "null communicator");
        c->timing = enable != 0;
    });
}

cad_status cad_comm_stats_read(cad_comm* c, cad_comm_stats* out) {
    return dp_guard([&] {
        if (!c || !out) throw DpError(CAD_ERR_INVALID, "null argument");
        DP_HIP(hipSetDevice(c->device));
        cad_comm_stats s = c->acc;
        for (int i = 0; i < c->ntimed; ++i) {
            const CommTimes& t = c->times[(size_t)i];
            DP_HIP(hipEventSynchronize(t.released));
            float exposed = 0.f, span = 0.f;
            DP_HIP(hipEventElapsedTime(&exposed, t.bwd_end, t.released));
            DP_HIP(hipEventElapsedTime(&span, t.ar_start, t.ar_end));
            s.exposed_ms += exposed;
            s.span_ms += span;
            ++s.timed_calls;
        }
        *out = s;
        c->acc = cad_comm_stats{};
        c->ntimed = 0;
    });
}

cad_status cad_comm_allreduce(cad_comm* c, float* buf, int64_t count, int op, void* stream) {
    return dp_guard([&] {
        if (!c || !buf || count < 0 || (op != CAD_REDUCE_SUM && op != CAD_REDUCE_MAX))
            throw DpError(CAD_ERR_INVALID, "bad all-reduce arguments");
        DP_HIP(hipSetDevice(c->device));
        DP_NCCL(ncclAllReduce(buf, buf, (size_t)count, ncclFloat32, op == CAD_REDUCE_SUM ? ncclSum : ncclMax, c->comm,
                              S(stream)));
    });
}

cad_status cad_comm_broadcast(cad_comm* c, float* buf, int64_t count, int root, void* stream) {
    return dp_guard([&] {
        if (!c || !buf || count < 0 || root < 0 || root >= c->nranks) throw DpError(CAD_ERR_INVALID, "bad broadcast arguments");
        DP_HIP(hipSetDevice(c->device));
        DP_NCCL(ncclBroadcast(buf, buf, (size_t)count, ncclFloat32, root, c->comm, S(stream)));
    });
}

cad_status cad_comm_broadcast_params(cad_unet* h, cad_comm* c, int root, void* stream) {
    return dp_guard([&] {
        float* p = nullptr;
        int64_t n = 0;
        if (cad_unet_flat(h, &p, nullptr, &n) != CAD_OK) throw DpError(CAD_ERR_INVALID, "cad_unet_flat failed");
        const cad_status st = cad_comm_broadcast(c, p, n, root, stream);
        if (st != CAD_OK) throw DpError(st, cad_last_error());
    });
}


cad_status cad_unet_backward_allreduce(cad_unet* h, cad_comm* c, const float* ddepth, int64_t bucket_elems,
                                       void* stream) {
    return dp_guard([&] {
        if (!h || !c || !ddepth) throw DpError(CAD_ERR_INVALID, "null argument");
        float* g = nullptr;
        if (cad_unet_flat(h, nullptr, &g, nullptr) != CAD_OK) throw DpError(CAD_ERR_INVALID, "cad_unet_flat failed");
        staged_backward_allreduce(
            c, g, cad_unet_num_stages(h), [&](int s, int64_t* o, int64_t* n) { return cad_unet_stage_grad_range(h, s, o, n); },
            [&](int s) { return cad_unet_backward_stage(h, s, ddepth, stream); }, bucket_elems, stream);
    });
}

cad_status cad_resunet_backward_allreduce(cad_resunet* h, cad_comm* c, const float* ddepth, int64_t bucket_elems,
                                          void* stream) {
    return dp_guard([&] {
        if (!h || !c || !ddepth) throw DpError(CAD_ERR_INVALID, "null argument");
        float* g = nullptr;
        if (cad_resunet_flat(h, nullptr, &g, nullptr) != CAD_OK) throw DpError(CAD_ERR_INVALID, "cad_resunet_flat failed");
        staged_backward_allreduce(
            c, g, cad_resunet_num_stages(h),
            [&](int s, int64_t* o, int64_t* n) { return cad_resunet_stage_grad_range(h, s, o, n); },
            [&](int s) { return cad_resunet_backward_stage(h, s, ddepth, stream); }, bucket_elems, stream);
    });
}

cad_status cad_geonet_backward_allreduce(cad_geonet* h, cad_comm* c, const float* ddepth, int64_t bucket_elems,
                                         void* stream) {
    return dp_guard([&] {
        if (!h || !c || !ddepth) throw DpError(CAD_ERR_INVALID, "null argument");
        float* g = nullptr;
        if (cad_geonet_flat(h, nullptr, &g, nullptr) != CAD_OK) throw DpError(CAD_ERR_INVALID, "cad_geonet_flat failed");
        staged_backward_allreduce(
            c, g, cad_geonet_num_stages(h),
            [&](int s, int64_t* o, int64_t* n) { return cad_geonet_stage_grad_range(h, s, o, n); },
            [&](int s) { return cad_geonet_backward_stage(h, s, ddepth, stream); }, bucket_elems, stream);
    });
}

cad_status cad_grad_allreduce(cad_unet* h, cad_comm* c, void* stream) {
    return dp_guard([&] {
        float* g = nullptr;
        int64_t n = 0;
        if (!h || !c || cad_unet_flat(h, nullptr, &g, &n) != CAD_OK) throw DpError(CAD_ERR_INVALID, "bad arguments");
        const cad_status st = cad_comm_allreduce(c, g, n, CAD_REDUCE_SUM, stream);
        if (st != CAD_OK) throw DpError(st, cad_last_error());
    });
}

}  // extern "C"

/*
 * cad.h — C ABI of libcad_hip.so, the MI355X (gfx950) implementation of the camera-aware depth
 * training step of RyoK3N/Camera-Aware-Neural-Networks-for-Few-View-Depth-Estimation.
 *
 * Boundary.  Each entry point replaces one reference interface on the hot path
 * (paths relative to the reference checkout):
 *   cad_unet_create / destroy       BaselineUNetImpl(in_channels, init_features, max_depth)
 *                                   src/models/baseline_unet.h:144-166 (+ TORCH_MODULE holder :208)
 *   cad_unet_count_parameters       BaselineUNetImpl::count_parameters        baseline_unet.h:200-206
 *   cad_unet_tensor_info/get/set    torch::nn::Module::named_parameters()/named_buffers() order and
 *                                   shapes (registration order, baseline_unet.h:20-30,53-56,79-81,
 *                                   147-165); used by torch::save / load and the trainer
 *   cad_unet_train                  Module::train()/eval()  (enhanced.h:259, :341)
 *   cad_unet_forward                BaselineUNetImpl::forward                 baseline_unet.h:174-195
 *   cad_unet_create_model           IntrinsicsConditionedUNetImpl(in, f, 4, max_depth)
 *                                   src/models/intrinsics_unet.h:137-200 (FiLMLayerImpl(4, C) per
 *                                   DoubleConv, src/layers/film_layer.h:47-72); CAD_MODEL_RAY_FILM =
 *                                   the config-3 composite with enc1 = RayEnhancedConv(3, f, 4, true)
 *                                   (src/models/geometry_aware_network.h:17-65)
 *   cad_unet_forward_cam            IntrinsicsConditionedUNetImpl::forward(x, intrinsics (B,4))
 *                                   intrinsics_unet.h:204-228 (+ RayEnhancedConvImpl::forward's
 *                                   cat(x, rays), geometry_aware_network.h:47-52)
 *   cad_camera_from_K               K (B,3,3) -> (B,4) [fx, fy, cx, cy] (the reference
 *                                   has no such code; train_main never builds camera vectors)
 *   cad_loss_create/forward_backward CombinedDepthLoss(si,grad,smooth,reproj) + forwardWithIntrinsics
 *                                   + the autograd backward of the loss       src/loss/depth_loss.h:366-433
 *   cad_loss_get_components         getComponentsWithIntrinsics               depth_loss.h:454-467
 *   cad_unet_backward[_stage]       loss.backward() through the U-Net         enhanced.h:297
 *   cad_clip_grad_norm              torch::nn::utils::clip_grad_norm_         enhanced.h:300-302
 *   cad_adam_create/step            torch::optim::Adam(AdamOptions(lr).weight_decay(wd)) / step()
 *                                   enhanced.h:97-101, :304
 *   cad_unet_flat                   flat gradient slab for the data-parallel RCCL all-reduce (new:
 *                                   the reference is single-device)
 *   cad_comm_* / cad_grad_allreduce / cad_unet_backward_allreduce
 *                                   data-parallel replicas over RCCL (new; SURVEY.md §8(b) proposal
 *                                   cad_grad_allreduce, §8(e) semantics; hardware.num_gpus /
 *                                   distributed keys of configs/train_config.yaml:178-183, which the
 *                                   reference parses but never uses)
 *   cad_loss_forward_backward_masked forwardWithIntrinsics(pred, gt, image, K, valid_mask)
 *                                   depth_loss.h:416-433 with the optional mask
 *   cad_depth_metrics               computeDepthMetrics (abs_rel ...)          enhanced.h:400-439
 *   cad_ray_directions              RayDirectionComputer::computeRayDirections
 *                                   src/preprocessing/ray_direction_computer.cpp:17-62
 *   cad_batcher_create/assemble     SunRGBDLoader::getSample's resizeSample + augmentSample
 *                                   (src/data/sunrgbd_loader.cpp:158-166, 352-489) and the trainer's
 *                                   batch torch::stack + .to(device) (enhanced.h:277-289), on device
 *   cad_aug_sampler_create/draw     augmentSample's random draws (sunrgbd_loader.cpp:352-443;
 *                                   AugmentationConfig sunrgbd_loader.h:30-42, rng_ seed :185)
 *   cad_op_*                        single operators of the step (conv, convT, BN, pool, ...), the
 *                                   ATen calls the reference dispatches
 *
 * Conventions: all tensor pointers are DEVICE pointers owned by the caller unless a handle owns
 * them; tensors crossing the boundary use the reference's NCHW fp32 layout (rgb (B,3,H,W), depth
 * (B,1,H,W), K (B,3,3) row-major).  Every call that launches work takes an explicit stream
 * (a hipStream_t passed as void*; NULL = default stream) and is asynchronous unless documented.
 * Status codes replace exceptions; cad_last_error() returns the thread-local message of the last
 * failing call.  Handles are not thread-safe: one handle per device per host thread.
 */
#ifndef CAD_CAD_H
#define CAD_CAD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CAD_ABI_VERSION 1

typedef enum {
    CAD_OK = 0,
    CAD_ERR_INVALID = 1, /* bad argument / shape */
    CAD_ERR_HIP = 2,     /* HIP runtime error */
    CAD_ERR_OOM = 3,     /* device allocation failed */
    CAD_ERR_STATE = 4    /* call out of order (e.g. backward before a train-mode forward) */
} cad_status;

typedef struct cad_unet cad_unet;
typedef struct cad_loss cad_loss;
typedef struct cad_adam cad_adam;

/* model families (cad_unet_create_model) */
#define CAD_MODEL_BASELINE 0        /* BaselineUNetImpl */
#define CAD_MODEL_INTRINSICS_FILM 1 /* IntrinsicsConditionedUNetImpl (camera_dim 4) */
#define CAD_MODEL_RAY_FILM 2        /* enc1 = RayEnhancedConv(3, f, 4, use_rays), FiLM blocks after */

typedef struct {
    int in_channels;   /* 3 */
    int init_features; /* f (64 default, 96 in train_config_production.yaml) */
    float max_depth;   /* 10.0 */
    int max_batch;     /* activation workspace is sized for this batch */
    int height;        /* H, W: must be divisible by 16 (the reference's pad branch is then a no-op) */
    int width;
} cad_unet_desc;

typedef struct {
    float lr;           /* optimization.learning_rate (1e-4) */
    float beta1, beta2; /* 0.9, 0.999 */
    float eps;          /* 1e-8 */
    float weight_decay; /* coupled L2 (torch::optim::Adam), 1e-5 */
} cad_adam_opts;

/* ---- library ---- */
int cad_abi_version(void);
/* GEMM engine of the conv3x3 / ConvTranspose contractions (forward, dgrad, wgrad):
 * CAD_GEMM_F32 = v_mfma_f32_32x32x2_f32 (exact fp32 fmaf chains); CAD_GEMM_S3 = fp32 operands split
 * exactly into three bf16 terms on the bf16 matrix cores, six products accumulated in fp32 (error
 * < 2^-23 |a b| per product: fp32 accuracy); CAD_GEMM_BF16 = operands rounded to bf16 (nearest
 * even), one product, fp32 accumulation — the bf16 arithmetic of BASELINE configs 3-5 (activations,
 * BatchNorm, loss and optimizer stay fp32).  Process-wide, default CAD_GEMM_S3; the env var
 * CAD_GEMM=f32|s3|bf16 sets the initial value. */
#define CAD_GEMM_F32 0
#define CAD_GEMM_S3 1
#define CAD_GEMM_BF16 2
cad_status cad_set_gemm_engine(int engine);
int cad_get_gemm_engine(void);
const char* cad_last_error(void);
/* Launch-level aliasing guard (csrc/host/alias.cpp): with mode 1 every instrumented launcher (the conv /
 * ConvT / dense GEMMs on every engine, the MX-fp8 GEMMs and quantiser, the BN / residual / pool / twin
 * passes) refuses a launch whose output byte range overlaps one of its inputs — CAD_ERR_INVALID, the
 * operands named in cad_last_error() — unless that pair is declared in place.  Default: the environment
 * (CAD_ALIAS_CHECK=1; tests/conftest.py sets it), else off.  Returns the previous mode. */
int cad_set_alias_check(int mode);
/* The guard's overlap rule on two row views (rows of ld elements of es bytes, columns [coff, coff+cols)):
 * 1 when they share a byte.  Host arithmetic only (no device). */
int cad_alias_views_overlap(const void* a, int64_t arows, int64_t ald, int64_t acoff, int64_t acols, int aes,
                            const void* b, int64_t brows, int64_t bld, int64_t bcoff, int64_t bcols, int bes);
cad_status cad_device_count(int* n);
cad_status cad_set_device(int device);
cad_status cad_stream_synchronize(void* stream);
/* device memory for callers without HIP headers (the C++ drop-in, the train CLI) */
cad_status cad_malloc(int device, int64_t bytes, void** out);
void cad_free(void* p);
/* kind: 0 host->device, 1 device->host, 2 device->device; synchronous when stream is NULL */
cad_status cad_memcpy(void* dst, const void* src, int64_t bytes, int kind, void* stream);

/* ---- model: BaselineUNetImpl ---- */
cad_status cad_unet_create(const cad_unet_desc* desc, int device, cad_unet** out); /* baseline */
cad_status cad_unet_create_model(const cad_unet_desc* desc, int model, int device, cad_unet** out);
int cad_unet_model(const cad_unet* h);
void cad_unet_destroy(cad_unet* h);
int64_t cad_unet_count_parameters(const cad_unet* h);
int cad_unet_num_params(const cad_unet* h);  /* tensors in named_parameters() */
int cad_unet_num_buffers(const cad_unet* h); /* float tensors in named_buffers() */
/* kind: 0 = parameter, 1 = buffer.  shape has up to 4 entries (reference layout). */
cad_status cad_unet_tensor_info(const cad_unet* h, int kind, int idx, const char** name, int* ndim,
                                int64_t shape[4]);
/* host <-> device copies in the REFERENCE layout (OIHW conv, (Cin,Cout,2,2) convT); synchronous */
cad_status cad_unet_set_tensor(cad_unet* h, int kind, int idx, const float* host, int64_t numel);
cad_status cad_unet_get_tensor(const cad_unet* h, int kind, int idx, float* host, int64_t numel);
cad_status cad_unet_get_grad(const cad_unet* h, int idx, float* host, int64_t numel);
cad_status cad_unet_train(cad_unet* h, int train); /* 1 = train(), 0 = eval() */
/* flat parameter / gradient slabs (internal packed layout; n = elements incl. alignment padding) */
cad_status cad_unet_flat(cad_unet* h, float** params, float** grads, int64_t* n);
/* switch the flat slabs to caller-owned device memory of cad_unet_flat()'s n floats each (e.g.
 * buffers a collective library registers); current parameter values are copied over.  The caller
 * keeps them alive for the handle's lifetime. */
cad_status cad_unet_use_external_slabs(cad_unet* h, float* params, float* grads);

/* forward: rgb (B,3,H,W) -> depth (B,1,H,W) in (0, max_depth).  B <= max_batch.
 * cad_unet_forward serves CAD_MODEL_BASELINE; the camera-conditioned models take cam4 (B,4)
 * [fx, fy, cx, cy] in pixels of the H x W input (normalised on device, intrinsics_unet.h:252-268;
 * RAY_FILM also derives the per-pixel rays from it).  Note FiLM's BatchNorm1d runs only for B > 1
 * (film_layer.h:85,91), in train and eval mode alike. */
cad_status cad_unet_forward(cad_unet* h, const float* rgb, float* depth, int B, void* stream);
cad_status cad_unet_forward_cam(cad_unet* h, const float* rgb, const float* cam4, float* depth, int B,
                                void* stream);
/* K (B,3,3) row-major -> cam4 (B,4) = [K00, K11, K02, K12] */
cad_status cad_camera_from_K(const float* K, int B, float* cam4, void* stream);

/* backward of the last train-mode forward given dL/ddepth; writes every parameter gradient.
 * Stage form (stage 0 .. cad_unet_num_stages()-1, in order) lets a caller overlap the gradient
 * all-reduce of finished stages with the rest of the backward. */
cad_status cad_unet_backward(cad_unet* h, const float* ddepth, void* stream);
int cad_unet_num_stages(const cad_unet* h);
cad_status cad_unet_backward_stage(cad_unet* h, int stage, const float* ddepth, void* stream);
/* [offset, offset+count) of the flat gradient slab completed by `stage` */
cad_status cad_unet_stage_grad_range(const cad_unet* h, int stage, int64_t* offset, int64_t* count);

/* clip_grad_norm_: total = ||prescale * g||_2; g *= prescale * min(1, max_norm / (total + 1e-6))
 * (the scaling is applied inside cad_adam_step; prescale = 1/world after a SUM all-reduce).
 * The total norm stays on device; cad_unet_last_grad_norm() fetches it (synchronises). */
cad_status cad_clip_grad_norm(cad_unet* h, float max_norm, float prescale, void* stream);
cad_status cad_unet_last_grad_norm(cad_unet* h, float* total_norm, void* stream);

/* ---- optimizer: torch::optim::Adam (coupled L2) over the model's flat slab ---- */
cad_status cad_adam_create(cad_unet* model, const cad_adam_opts* opts, cad_adam** out);
void cad_adam_destroy(cad_adam* a);
cad_status cad_adam_step(cad_adam* a, void* stream); /* consumes the clip coefficient */
cad_status cad_adam_set_lr(cad_adam* a, float lr);
int64_t cad_adam_step_count(const cad_adam* a);
/* optimizer state for checkpoint / resume: device pointers to the m and v slabs (cad_unet_flat's n
 * floats each, same packed layout as the parameters) and the step counter */
cad_status cad_adam_state(cad_adam* a, float** m, float** v);
cad_status cad_adam_set_step_count(cad_adam* a, int64_t step);

/* ---- checkpoints in the reference's format: torch::save(model_, path) / torch::load(model, path)
 * (tensorboard_trainer_enhanced.h:656-662; production_trainer.h:323-330 writes final_model.pt).
 * cad_unet_save_torch writes the TorchScript zip archive LibTorch's OutputArchive produces for the
 * module (every parameter and buffer under its named_parameters()/named_buffers() name, BatchNorm
 * num_batches_tracked included, parameterless submodules such as the encoders' MaxPool2d kept), so
 * torch::load of the reference model reads it; cad_unet_load_torch reads such an archive (from the
 * reference or from us) into the model: every model tensor must be present with its shape (extra
 * archive entries are ignored, as torch::load ignores them).  Synchronous. */
cad_status cad_unet_save_torch(cad_unet* h, const char* path);
cad_status cad_unet_load_torch(cad_unet* h, const char* path);
/* BatchNorm num_batches_tracked: train-mode forwards since creation (or the loaded value) */
int64_t cad_unet_num_batches_tracked(const cad_unet* h);

/* host-only archive I/O underneath (no device needed).  Entries are written in the order given:
 * a module's parameters (kind 0), then its buffers (kind 1), then its children in first-appearance
 * order; kind 2 declares a parameterless submodule (e.g. "enc2.pool") at its registration position. */
#define CAD_DTYPE_F32 0
#define CAD_DTYPE_I64 1
#define CAD_DTYPE_F64 2
#define CAD_DTYPE_F16 3
#define CAD_DTYPE_BF16 4
#define CAD_DTYPE_I32 5
typedef struct {
    const char* name;  /* dotted path, e.g. "enc1.bn1.running_mean" */
    int kind;          /* 0 parameter, 1 buffer, 2 empty submodule */
    int dtype;         /* CAD_DTYPE_* */
    int ndim;          /* 0..8 (0 = scalar) */
    int64_t shape[8];
    const void* data;  /* contiguous host data */
} cad_archive_entry;
cad_status cad_archive_write(const char* path, const cad_archive_entry* entries, int n);
/* reader: a data-only pickle interpreter (nothing named in the file is executed) over torch::save
 * module archives and Python torch.save state dicts; tensors are listed under dotted names */
typedef struct cad_archive cad_archive;
cad_status cad_archive_open(const char* path, cad_archive** out);
void cad_archive_close(cad_archive* a);
int cad_archive_count(const cad_archive* a);
int cad_archive_find(const cad_archive* a, const char* name); /* -1 if absent */
cad_status cad_archive_info(const cad_archive* a, int i, const char** name, int* dtype, int* ndim, int64_t shape[8]);
cad_status cad_archive_read(const cad_archive* a, int i, void* dst, int64_t bytes); /* raw, in its dtype */

/* ---- data-parallel gradient exchange: RCCL over xGMI, one process per GPU (new: the reference is
 * single-device).  Semantics: every replica runs the same step on
 * its own shard of the global batch (BN statistics and loss masks per replica); the gradient slab is
 * SUM-all-reduced and the 1/world mean folded into cad_clip_grad_norm(.., prescale = 1/world);
 * clip and Adam are then identical on every replica. ---- */
typedef struct cad_comm cad_comm;
#define CAD_COMM_ID_BYTES 128
#define CAD_REDUCE_SUM 0
#define CAD_REDUCE_MAX 1
/* rank 0 draws the communicator id (ncclGetUniqueId) and hands its bytes to every rank */
cad_status cad_comm_get_unique_id(uint8_t id[CAD_COMM_ID_BYTES]);
/* collective: every rank of the job calls it with the same id (ncclCommInitRank) */
cad_status cad_comm_create(const uint8_t id[CAD_COMM_ID_BYTES], int nranks, int rank, int device, cad_comm** out);
void cad_comm_destroy(cad_comm* c);
int cad_comm_rank(const cad_comm* c);
int cad_comm_size(const cad_comm* c);
/* in-place fp32 all-reduce / broadcast on `stream` (e.g. loss and metric scalars, initial weights) */
cad_status cad_comm_allreduce(cad_comm* c, float* buf, int64_t count, int op, void* stream);
cad_status cad_comm_broadcast(cad_comm* c, float* buf, int64_t count, int root, void* stream);
/* the flat parameter slab of `h` from rank `root` (identical replicas at start / after a resume) */
cad_status cad_comm_broadcast_params(cad_unet* h, cad_comm* c, int root, void* stream);
/* SUM all-reduce of the whole gradient slab after a backward (no overlap; SURVEY §8(b)'s proposal) */
cad_status cad_grad_allreduce(cad_unet* h, cad_comm* c, void* stream);
/* loss.backward() with the exchange overlapped: every backward stage is enqueued on `stream`; as soon
 * as the stages of a bucket (>= bucket_elems floats, decoder first, cad_plan_grad_buckets) are
 * enqueued, its SUM all-reduce is issued on the communicator's stream behind an event, so RCCL runs
 * while the remaining dgrad/wgrad kernels do; `stream` finally waits for every all-reduce. */
cad_status cad_unet_backward_allreduce(cad_unet* h, cad_comm* c, const float* ddepth, int64_t bucket_elems,
                                       void* stream);
/* Exchange accounting of the *_backward_allreduce calls (new; no reference counterpart).  With timing
 * on, each call records HIP timing events: on the compute stream after its last backward kernel and
 * again once that stream has waited for the last all-reduce (the difference is the exposed, i.e.
 * non-overlapped, exchange time), and on the communicator's stream around its all-reduces (the span
 * from the first bucket's start to the last bucket's end).  cad_comm_stats waits for the recorded
 * events, returns the sums since the last read (or since timing was enabled) and resets them.  At most
 * 256 calls are timed between reads (later ones are counted in `calls`/`bytes` only). */
typedef struct cad_comm_stats {
    int64_t calls;          /* backward_allreduce calls */
    int64_t timed_calls;    /* calls whose events were recorded */
    int64_t buckets;        /* all-reduces issued */
    int64_t bytes;          /* bytes all-reduced (fp32 SUM, in place) */
    double exposed_ms;      /* sum over timed calls: last backward kernel -> compute stream released */
    double span_ms;         /* sum over timed calls: first all-reduce start -> last all-reduce end */
} cad_comm_stats;
cad_status cad_comm_set_timing(cad_comm* c, int enable);
cad_status cad_comm_stats_read(cad_comm* c, cad_comm_stats* out);
/* the bucket plan (host only): consecutive backward stages [stage_off, +stage_cnt) grouped greedily
 * into contiguous buckets of >= bucket_elems floats (the last takes the rest).  Writes up to nstages
 * buckets (nullable outputs); returns the bucket count, or -1 on bad input. */
int cad_plan_grad_buckets(const int64_t* stage_off, const int64_t* stage_cnt, int nstages, int64_t bucket_elems,
                          int64_t* bucket_off, int64_t* bucket_cnt, int* bucket_last_stage);
/* host only (no device): the flat gradient slab layout of a model family — backward stage count (at
 * most 16) and each stage's [offset, offset+count) — as cad_unet_stage_grad_range reports it */
cad_status cad_model_grad_layout(int model, int in_channels, int init_features, int* nstages, int64_t stage_off[16],
                                 int64_t stage_cnt[16], int64_t* n_flat);

/* ---- loss: CombinedDepthLoss ---- */
cad_status cad_loss_create(float si_weight, float grad_weight, float smooth_weight, float reproj_weight,
                           int max_batch, int height, int width, int device, cad_loss** out);
void cad_loss_destroy(cad_loss* l);
/* forwardWithIntrinsics + backward: loss5 (device, 5 floats) = {total, si, grad, smooth, reproj};
 * dpred (device, B*H*W) = dL/dpred.  K (B,3,3) row-major. */
cad_status cad_loss_forward_backward(cad_loss* l, const float* pred, const float* gt, const float* rgb,
                                     const float* K, int B, float* loss5, float* dpred, void* stream);
/* the same with forwardWithIntrinsics' optional valid_mask (depth_loss.h:416-433): mask (device,
 * B*H*W bytes, nonzero = valid) replaces the default gt > 1e-6 mask of the scale-invariant and
 * reprojection terms (:38-40, :320-322); the gradient-matching term ignores it like the reference
 * (:137) and smoothness never takes one (:189).  mask == NULL: cad_loss_forward_backward. */
cad_status cad_loss_forward_backward_masked(cad_loss* l, const float* pred, const float* gt, const float* rgb,
                                            const float* K, const uint8_t* mask, int B, float* loss5, float* dpred,
                                            void* stream);
/* getComponentsWithIntrinsics: host copy of {total, si, grad, smooth, reproj} of the last call */
cad_status cad_loss_get_components(cad_loss* l, float out5[5], void* stream);

/* ---- metrics (computeDepthMetrics) on host-visible results: abs_rel etc. per sample, averaged */
cad_status cad_depth_metrics(const float* pred, const float* gt, int B, int H, int W, float out7[7],
                             void* stream);

/* ---- conditioning: per-pixel unit ray directions (B,3,H,W) from K (B,3,3) ---- */
cad_status cad_ray_directions(const float* K, int B, int H, int W, float* rays, void* stream);

/* ---- batch assembly on device: decoded samples -> the step's (B,3,H,W) rgb, (B,1,H,W) depth,
 * (B,3,3) K.  Per sample: rgb = u8/255, depth = u16 * depth_scale, resized to H x W (rgb bilinear,
 * align_corners = false; depth nearest; K scaled), then — when aug is set — crop (window clamped to
 * the image like a torch Slice, K's principal point shifted), horizontal flip (cx = W - cx - 1),
 * colour jitter clamp(rgb * contrast + brightness - 1, 0, 1), and the resize back to H x W. */
typedef struct {
    const uint8_t* rgb;     /* device: decoded image, HWC u8, h0 x w0 x 3 */
    const uint16_t* depth;  /* device: decoded depth, HW u16 */
    int h0, w0;
    int bgr;                /* 1: rgb is in OpenCV BGR order (loadRGB's cvtColor happens here) */
    float depth_scale;      /* metres per unit: 1/1000 (loadDepth) */
    float K[9];             /* host: the sample's intrinsics, 3x3 row-major */
    int aug;                /* 0: resize only (validation / augmentation off) */
    int crop;               /* applyCrop with crop_scale, crop_x, crop_y (on the resized image) */
    float crop_scale;
    int crop_x, crop_y;
    int flip;               /* applyHorizontalFlip */
    int jitter;             /* applyColorJitter with brightness, contrast */
    float brightness, contrast;
    int dh0, dw0;           /* depth map size when it differs from the image's (0: h0 x w0) */
} cad_sample;
typedef struct cad_batcher cad_batcher;
cad_status cad_batcher_create(int max_batch, int height, int width, int device, cad_batcher** out);
void cad_batcher_destroy(cad_batcher* b);
/* asynchronous on `stream`; samples[] is read before the call returns */
cad_status cad_batcher_assemble(cad_batcher* b, const cad_sample* samples, int B, float* rgb, float* depth,
                                float* K, void* stream);

typedef struct { /* AugmentationConfig (sunrgbd_loader.h:30-42) */
    int enable_random_crop;
    float crop_scale_min, crop_scale_max; /* 0.7, 1.0 */
    int enable_horizontal_flip;
    float horizontal_flip_prob; /* 0.5 */
    int enable_color_jitter;
    float brightness_delta, contrast_delta; /* 0.2, 0.2 */
} cad_aug_config;
typedef struct cad_aug_sampler cad_aug_sampler;
/* std::mt19937 seeded like the loader's rng_ (config.random_seed) */
cad_status cad_aug_sampler_create(const cad_aug_config* cfg, uint32_t seed, cad_aug_sampler** out);
void cad_aug_sampler_destroy(cad_aug_sampler* s);
/* fills sample->aug/crop/flip/jitter fields with augmentSample's draws, in its order, for an image
 * already resized to height x width */
cad_status cad_aug_sampler_draw(cad_aug_sampler* s, int height, int width, cad_sample* sample);

/* ---- the loader: SunRGBDLoader's manifest + decoding (src/data/sunrgbd_loader.cpp:39-102, 221-275)
 * and a prefetch ring into the batcher.  cad_dataset_open reads the JSON manifest: "images" entries
 * with valid == true, a sensor_type in sensors[] (NULL/0: kv1, kv2, realsense, xtion — the loader's
 * default) and an existing <path>/intrinsics.txt, in manifest order (paths relative to the working
 * directory, as in the reference).  A sample decodes <path>/image/<first .jpg|.png|.ppm> as RGB u8
 * and <path>/depth/<first .png|.pgm> as u16 (16-bit: metres = value / 1000; 8-bit: value), PNG and
 * binary PNM, and baseline / extended-sequential / progressive Huffman JPEG (csrc/host/jpeg.cpp:
 * libjpeg-turbo's default decompression — ISLOW IDCT, fancy upsampling, jdcolor.c YCbCr->RGB —
 * restated bit for bit; arithmetic / lossless / 12-bit / CMYK JPEGs and progressions cut short (which
 * libjpeg-turbo block-smooths) fail with a message). */
typedef struct cad_dataset cad_dataset;
/* decode a JPEG file held in memory (what cv::imread(IMREAD_COLOR) decodes for the loader,
 * sunrgbd_loader.cpp:86,222, before its BGR order): height x width x channels u8 samples (channels 1
 * gray or 3 RGB) into out (out == NULL: dimensions only) */
cad_status cad_jpeg_decode(const uint8_t* data, int64_t size, uint8_t* out, int64_t cap, int* height, int* width,
                           int* channels);
typedef struct {
    int h0, w0;        /* rgb size */
    int dh0, dw0;      /* depth size */
    float depth_scale; /* metres per depth unit */
    float K[9];        /* intrinsics.txt, row-major */
} cad_decoded_info;
cad_status cad_dataset_open(const char* manifest_path, const char* const* sensors, int n_sensors, cad_dataset** out);
/* n procedurally generated decoded samples of height x width (the synthetic dataset) */
cad_status cad_dataset_synthetic(int64_t n, int height, int width, uint32_t seed, cad_dataset** out);
void cad_dataset_destroy(cad_dataset* d);
int64_t cad_dataset_size(const cad_dataset* d);
const char* cad_dataset_image_dir(const cad_dataset* d, int64_t i); /* NULL for synthetic */
/* host decode of sample i into rgb (h0*w0*3 bytes) and depth (dh0*dw0 u16); either may be NULL to
 * query info only */
cad_status cad_dataset_read(const cad_dataset* d, int64_t i, uint8_t* rgb, int64_t rgb_cap, uint16_t* depth,
                            int64_t depth_cap, cad_decoded_info* info);
/* Prefetch ring: `threads` host workers decode up to `slots` (>= 2) batches ahead into pinned
 * buffers; each batch is uploaded on the loader's copy stream and assembled on the caller's stream
 * by a cad_batcher (resize; with aug != NULL, augmentSample's draws from a mt19937 seeded `seed`,
 * drawn in sample order).  The dataset must outlive the loader. */
typedef struct cad_loader cad_loader;
cad_status cad_loader_create(const cad_dataset* ds, int batch, int height, int width, const cad_aug_config* aug,
                             uint32_t seed, int threads, int slots, int device, cad_loader** out);
void cad_loader_destroy(cad_loader* L);
/* the epoch's sample order (NULL: 0..n-1); batches of `batch`, the last one partial (trainEpoch) */
cad_status cad_loader_start_epoch(cad_loader* L, const int64_t* order, int64_t n);
/* the next batch into rgb (B,3,H,W), depth (B,1,H,W), K (B,3,3) device fp32, asynchronously on
 * `stream`; returns its size B (0 at the end of the epoch, -1 on error: cad_last_error()) */
int cad_loader_next(cad_loader* L, float* rgb, float* depth, float* K, void* stream);

/* ---- debugging: synchronous host copy of an internal NHWC activation buffer by name
 * ("x0", "cat<l>", "dcat<l>", "pool<l>", "dout<l>", "bott", "Sa", "Sb", "Sc",
 *  "enc<l>.y1|a1|y2", "dec<l>.y1|a1|y2"); numel = rows*channels of the last forward's batch.
 * Returns the element count (host may be NULL to query), or -1 for an unknown name — and, on the
 * bf16 engine (pre-split operands), for the buffers whose fp32 copy that path does not write
 * ("Sb", "bott", "pool<l>", "dout1..3", every block's a1); cad_last_error() says which. */
int64_t cad_unet_debug_buffer(cad_unet* h, const char* name, float* host, int64_t numel);

/* ---- launch profiler: HIP events around every MFMA GEMM launch on its own stream ---- */
cad_status cad_profile_enable(int on);
cad_status cad_profile_reset(void);
/* time only the launches of the kernel named kernel_name (as the report names it); NULL or "": all */
cad_status cad_profile_only(const char* kernel_name);
/* writes a JSON array [{"name","launches","ms","gflop"}...] into buf (synchronises); returns the
 * length needed including the terminator */
int cad_profile_report(char* buf, int cap);

/* ---- operator-level entry points (NHWC fp32; ld = floats between pixels, coff = channel offset) */
cad_status cad_op_conv3x3_fwd(const float* x, int64_t ldx, int xcoff, int cin, const float* w_ohwi,
                              int cout, float* y, int64_t ldy, int ycoff, int B, int H, int W,
                              void* stream);
cad_status cad_op_conv3x3_dgrad(const float* dz, int cout, const float* w_ohwi, int cin, float* dx,
                                int64_t lddx, int B, int H, int W, void* stream);
cad_status cad_op_conv3x3_wgrad(const float* dz, int cout, const float* x, int64_t ldx, int xcoff, int cin,
                                float* dw_ohwi, int B, int H, int W, void* stream);
/* the bf16 engine's weight gradient on pre-split bf16 NHWC operands (the twins the engine stores):
 * dz rows of lddz bf16, x rows of ldx bf16 at channel offset xcoff (% 8); fp32 OHWI result.  Window
 * kernel when cout, cin % 64 == 0 and W % 16 == 0, the im2col GEMM otherwise.  Requires
 * cad_set_gemm_engine(CAD_GEMM_BF16). */
cad_status cad_op_conv3x3_wgrad_bf16(const void* dz, int64_t lddz, int cout, const void* x, int64_t ldx, int xcoff,
                                     int cin, float* dw_ohwi, int B, int H, int W, void* stream);
/* the bf16 engine's 3x3 convolution forward / input gradient on pre-split bf16 NHWC operands (the twins
 * the engine stores), fp32 OHWI weights rounded to bf16 inside (the dgrad repacks them first):
 * window kernels (gemm_win.hpp) when the shape allows, the im2col GEMM otherwise.  y / dx: fp32 rows, or
 * bf16 rows with y_bf16 / dx_bf16.  with_stats: the forward also forms its BN tile partials (the
 * EpiStoreStats epilogue; the partials are discarded — timing and coverage).  Requires
 * cad_set_gemm_engine(CAD_GEMM_BF16); the bf16 forms of baseline_unet.h:32-42 DoubleConv's convs. */
cad_status cad_op_conv3x3_fwd_bf16(const void* x, int64_t ldx, int xcoff, int cin, const float* w_ohwi, int cout,
                                   void* y, int64_t ldy, int ycoff, int y_bf16, int with_stats, int B, int H, int W,
                                   void* stream);
cad_status cad_op_conv3x3_dgrad_bf16(const void* dz, int64_t lddz, int cout, const float* w_ohwi, int cin, void* dx,
                                     int64_t lddx, int dx_bf16, int B, int H, int W, void* stream);
cad_status cad_op_convT_fwd(const float* x, int cin, const float* w_iqo, const float* bias, int cout,
                            float* y, int64_t ldy, int ycoff, int B, int H, int W, void* stream);
/* the bf16 engine's ConvTranspose2d(k2, s2) forward (baseline_unet.h:91 `up`) on a pre-split bf16 NHWC
 * input (rows of ldx, channel offset xcoff), fp32 [ci][dy][dx][co] weights rounded to bf16 inside:
 * y (bf16 rows of ldy at channel offset ycoff, the decoder concat's up half) = x * w + bias, pixel-
 * shuffled.  Requires cad_set_gemm_engine(CAD_GEMM_BF16). */
cad_status cad_op_convT_fwd_bf16(const void* x, int64_t ldx, int xcoff, int cin, const float* w_iqo,
                                 const float* bias, int cout, void* y, int64_t ldy, int ycoff, int B, int H, int W,
                                 void* stream);
cad_status cad_op_convT_dgrad(const float* g, int64_t ldg, int gcoff, int cout, const float* w_iqo, int cin,
                              float* dx, int B, int H, int W, void* stream);
cad_status cad_op_convT_wgrad(const float* x, int cin, const float* g, int64_t ldg, int gcoff, int cout,
                              float* dw_iqo, int B, int H, int W, void* stream);
cad_status cad_op_maxpool_fwd(const float* x, int64_t ldx, int C, int B, int H, int W, float* out,
                              uint8_t* idx, void* stream);

/* MX-fp8 operands (OCP MXFP8 E4M3, one E8M0 scale per 32 consecutive k; the config-5 network's forward
 * conv-GEMMs, kernels.hpp Mx8): q = element bytes [rows][ldq], s = scale bytes [rows][ldq / 32],
 * ldq % 128 == 0.  quantize: rows [qcoff, qcoff + C) of (q, s) from src rows [scoff, scoff + C)
 * (fp32, or bf16 when src_bf16), C % 32 == 0. */
cad_status cad_op_mx8_quantize(const void* src, int src_bf16, int64_t lds, int scoff, int C, int64_t M, void* q,
                               void* s, int64_t ldq, int qcoff, void* stream);
/* y[m][n] (fp32, dense [M][N]) = sum_k x[m][k] w[n][k] on MX operands; K % 128 == 0, N % 64 == 0 */
cad_status cad_op_dense_x8(const void* xq, const void* xs, int64_t ldx, int K, const void* wq, const void* ws,
                           int64_t ldw, int N, float* y, int64_t M, void* stream);
/* y[pix][co] (fp32, dense [B*H*W][cout]) = conv3x3(x) on MX operands: x rows [pix][ldx] (cin channels),
 * w rows [cout][ldw] in (tap, ci) order (ldw >= 9 cin); cin % 64, cout % 64 and a window block width
 * dividing W (the window kernel), else CAD_ERR_INVALID */
cad_status cad_op_conv3x3_x8(const void* xq, const void* xs, int64_t ldx, int cin, const void* wq, const void* ws,
                             int64_t ldw, int cout, float* y, int B, int H, int W, void* stream);

/* ---- config-5 network (BASELINE configs[4]): ResNet-50 encoder + U-Net decoder, bf16 operands ----
 * No reference counterpart: architecture in resunet.cpp / DESIGN.md §9;
 * torchvision ResNet-50 parameter names under "encoder.", decoder "dec4".."dec0", "out_conv".
 * Same life cycle as cad_unet: forward (train: BN batch statistics), backward (dL/ddepth), clip,
 * Adam (moments owned by the model). height / width multiples of 32. */
typedef struct cad_resunet cad_resunet;
typedef struct {
    int in_channels;   /* 3 */
    int max_batch;
    int height, width;
    float max_depth;
} cad_resunet_desc;
cad_status cad_resunet_create(const cad_resunet_desc* d, int device, cad_resunet** out);
void cad_resunet_destroy(cad_resunet* h);
int64_t cad_resunet_count_parameters(const cad_resunet* h);
int cad_resunet_num_tensors(const cad_resunet* h, int kind);   /* 0 parameters, 1 buffers */
cad_status cad_resunet_tensor_info(const cad_resunet* h, int kind, int idx, const char** name, int* ndim,
                                   int64_t shape[4]);
cad_status cad_resunet_set_tensor(cad_resunet* h, int kind, int idx, const float* host, int64_t numel);
cad_status cad_resunet_get_tensor(const cad_resunet* h, int kind, int idx, float* host, int64_t numel);
cad_status cad_resunet_get_grad(const cad_resunet* h, int idx, float* host, int64_t numel);
cad_status cad_resunet_train(cad_resunet* h, int train);
/* MX-fp8 forward conv-GEMMs (configs[4] "bf16 with fp8 MFMA conv-GEMM"): on = 1 runs
 * every eligible forward contraction (the 1x1 / im2col GEMMs with K % 128 == 0, the 3x3 window
 * convolutions with cin % 64 == 0) on OCP MXFP8 E4M3 operands with one E8M0 scale per 32 channels
 * (v_mfma_scale_f32_32x32x64_f8f6f4, fp32 accumulation); the stem, ConvTs, the backward (dgrad,
 * wgrad) and everything else stay as on 0 (bf16 operands).  Default 0.  fp8_units: how many
 * convolutions are eligible. */
cad_status cad_resunet_set_fp8(cad_resunet* h, int on);
int cad_resunet_fp8_units(const cad_resunet* h);
cad_status cad_resunet_flat(cad_resunet* h, float** params, float** grads, int64_t* n);
cad_status cad_resunet_forward(cad_resunet* h, const float* rgb, float* depth, int B, void* stream);
cad_status cad_resunet_backward(cad_resunet* h, const float* ddepth, void* stream);
/* staged backward (decoder first; stage s writes only the gradients in its flat-slab range, ranges
 * decreasing with s) and the overlapped data-parallel exchange over it (cad_unet_backward_allreduce's
 * semantics: SUM buckets of >= bucket_elems floats on the communicator's stream) */
/* Test hook: a buffer of the last train-mode forward as fp32 rows — "y:<conv>" (stored pre-BN output,
   bf16 widened), "scale:<bn>" / "shift:<bn>" (BN-apply coefficients), "out:<block>" (block output:
   "encoder.layer<L>.<i>", "encoder.stem", "dec<l>"), "cat:dec<l>" (a decoder's bf16 input [skip, up]).
   Returns the element count, -1 if unknown. */
int64_t cad_resunet_debug_buffer(cad_resunet* h, const char* name, float* host, int64_t numel);
int cad_resunet_num_stages(const cad_resunet* h);
/* host only (no device): the stage count (23) and each stage's [offset, offset+count), as
 * cad_resunet_stage_grad_range reports them, and the slab size */
cad_status cad_resunet_grad_layout(int* nstages, int64_t stage_off[32], int64_t stage_cnt[32], int64_t* n_flat);
cad_status cad_resunet_stage_grad_range(const cad_resunet* h, int stage, int64_t* offset, int64_t* count);
cad_status cad_resunet_backward_stage(cad_resunet* h, int stage, const float* ddepth, void* stream);
cad_status cad_resunet_backward_allreduce(cad_resunet* h, cad_comm* c, const float* ddepth, int64_t bucket_elems,
                                          void* stream);
cad_status cad_resunet_clip_grad_norm(cad_resunet* h, float max_norm, float prescale, void* stream);
cad_status cad_resunet_last_grad_norm(cad_resunet* h, float* total_norm, void* stream);
cad_status cad_resunet_adam_step(cad_resunet* h, float lr, float beta1, float beta2, float eps, float weight_decay,
                                 void* stream);

/* ---- geometry-aware family, src/models/geometry_aware_network.h ----
 *   cad_geonet_create (CAD_GEONET_FULL)   GeometryAwareNetworkImpl(3, f, 4, max_depth, use_pcl,
 *                                         use_attention)  geometry_aware_network.h:201-278
 *   cad_geonet_create (CAD_GEONET_LIGHT)  LightweightGeometryNetworkImpl(3, f, 4, max_depth)  :355-383
 *   cad_geonet_forward                    GeometryAwareNetworkImpl::forward(rgb, ray_directions,
 *                                         camera_intrinsics (B,4) [fx, fy, cx, cy])  :289-318 / :385-402
 *     (RayEnhancedConvImpl :17-65, GeometryEncoderBlockImpl :74-104, GeometryDecoderBlockImpl
 *      :112-170, CBAMImpl spatial_attention.h:142-191, PerspectiveCorrectionLayerImpl pcl_layer.h:29-181)
 * rgb, rays (B,3,H,W) NCHW device fp32; depth (B,1,H,W).  Parameter / buffer names and order are the
 * reference module's named_parameters() / named_buffers() (float buffers).  Same life cycle as
 * cad_resunet.  H, W multiples of 32 (FULL, 5 pools) or 16 (LIGHT). */
#define CAD_GEONET_FULL 0
#define CAD_GEONET_LIGHT 1
typedef struct cad_geonet cad_geonet;
typedef struct {
    int variant;        /* CAD_GEONET_FULL / CAD_GEONET_LIGHT */
    int in_channels;    /* 3 */
    int init_features;  /* 64 (FULL default), 32 (LIGHT default) */
    int camera_dim;     /* 4 */
    float max_depth;    /* 10.0 */
    int use_pcl;        /* FULL only (LIGHT: always 1) */
    int use_attention;  /* FULL only (LIGHT: always 1) */
    int max_batch;
    int height, width;
} cad_geonet_desc;
cad_status cad_geonet_create(const cad_geonet_desc* d, int device, cad_geonet** out);
void cad_geonet_destroy(cad_geonet* h);
int64_t cad_geonet_count_parameters(const cad_geonet* h);
int cad_geonet_num_tensors(const cad_geonet* h, int kind);   /* 0 parameters, 1 buffers */
cad_status cad_geonet_tensor_info(const cad_geonet* h, int kind, int idx, const char** name, int* ndim,
                                  int64_t shape[4]);
cad_status cad_geonet_set_tensor(cad_geonet* h, int kind, int idx, const float* host, int64_t numel);
cad_status cad_geonet_get_tensor(const cad_geonet* h, int kind, int idx, float* host, int64_t numel);
cad_status cad_geonet_get_grad(const cad_geonet* h, int idx, float* host, int64_t numel);
cad_status cad_geonet_train(cad_geonet* h, int train);
cad_status cad_geonet_flat(cad_geonet* h, float** params, float** grads, int64_t* n);
cad_status cad_geonet_forward(cad_geonet* h, const float* rgb, const float* rays, const float* cam4, float* depth,
                              int B, void* stream);
cad_status cad_geonet_backward(cad_geonet* h, const float* ddepth, void* stream);
/* staged backward and the overlapped data-parallel exchange (as cad_resunet_*) */
int cad_geonet_num_stages(const cad_geonet* h);
/* host only (no device): the stage layout of the network `d` describes (as cad_resunet_grad_layout) */
cad_status cad_geonet_grad_layout(const cad_geonet_desc* d, int* nstages, int64_t stage_off[16], int64_t stage_cnt[16],
                                  int64_t* n_flat);
cad_status cad_geonet_stage_grad_range(const cad_geonet* h, int stage, int64_t* offset, int64_t* count);
cad_status cad_geonet_backward_stage(cad_geonet* h, int stage, const float* ddepth, void* stream);
cad_status cad_geonet_backward_allreduce(cad_geonet* h, cad_comm* c, const float* ddepth, int64_t bucket_elems,
                                         void* stream);
cad_status cad_geonet_clip_grad_norm(cad_geonet* h, float max_norm, float prescale, void* stream);
cad_status cad_geonet_last_grad_norm(cad_geonet* h, float* total_norm, void* stream);
cad_status cad_geonet_adam_step(cad_geonet* h, float lr, float beta1, float beta2, float eps, float weight_decay,
                                void* stream);
/* BatchNorm num_batches_tracked: film = 0 the BatchNorm2d layers, 1 FiLM's BatchNorm1d (B > 1 only) */
int64_t cad_geonet_num_batches_tracked(const cad_geonet* h, int film);
/* operator-level entry points (tests; state allocated per call): one CBAMImpl forward + backward
 * (spatial_attention.h:142-191) / one PerspectiveCorrectionLayerImpl forward + backward (pcl_layer.h:
 * 76-178) on device NHWC tensors [B*H*W][C]; params / grads packed in registration order
 * (CBAM: fc1.w [C/16][C], fc1.b, fc2.w [C][C/16], fc2.b, spatial conv.w [2][7][7]; PCL: loc_fc1.w
 * [128][C+4], loc_fc1.b, loc_fc2.w [128][128], loc_fc2.b, fc_transform.w [6][128], fc_transform.b);
 * g = gradient of the output; camn (B,4) the normalised intrinsics; theta (nullable) <- (B,2,3) */
cad_status cad_op_cbam(const float* x, const float* g, const float* params, int B, int H, int W, int C, float* out,
                       float* dx, float* grads, void* stream);
cad_status cad_op_pcl(const float* u, const float* camn, const float* g, const float* params, int B, int H, int W,
                      int C, float* out, float* du, float* grads, float* theta, void* stream);
/* test hook: buffer of the last step ("cat<l>", "dcat<l>", "x<l>", "u<l>", "z<l>"; NHWC rows) -> host;
 * returns the element count (host NULL: count only) or -1 */
int64_t cad_geonet_debug_buffer(cad_geonet* h, const char* name, float* host, int64_t numel);

#ifdef __cplusplus
}
#endif
#endif /* CAD_CAD_H */

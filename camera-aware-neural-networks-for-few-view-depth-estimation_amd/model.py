"""Python host mirror of the reference's hot-path operator API, on libcad_hip.so.

Class and method names follow the reference so that a caller (and the parity tests) read like
the reference's own code:

  BaselineUNet            BaselineUNetImpl           src/models/baseline_unet.h:122-208
  IntrinsicsConditionedUNet IntrinsicsConditionedUNetImpl src/models/intrinsics_unet.h:137-270
  RayConditionedUNet      config-3 composite: enc1 = RayEnhancedConv (geometry_aware_network.h:17-65),
                          FiLM blocks after (intrinsics_unet.h:16-113)
  CombinedDepthLoss       CombinedDepthLoss          src/loss/depth_loss.h:366-479
  Adam                    torch::optim::Adam         (options built at tensorboard_trainer_enhanced.h:97-101)
  clip_grad_norm_         torch::nn::utils::clip_grad_norm_ (enhanced.h:300-302)
  Trainer.train_step      TensorBoardTrainerEnhanced::trainEpoch body, enhanced.h:287-304

torch is used only as device-memory / stream / torch.distributed plumbing: every computation on the
path runs in the HIP kernels behind the C ABI.  Tensors are torch CUDA (HIP) tensors in the
reference's NCHW fp32 layout.
"""
from __future__ import annotations

import ctypes as C
from collections import OrderedDict

import numpy as np
import torch

from . import _abi
from ._abi import check


def _stream(device=None):
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _ptr(t: torch.Tensor):
    assert t.is_cuda and t.is_contiguous() and t.dtype == torch.float32, "expected contiguous fp32 device tensor"
    return C.c_void_p(t.data_ptr())


MODEL_BASELINE, MODEL_INTRINSICS_FILM, MODEL_RAY_FILM = 0, 1, 2   # CAD_MODEL_* of cad.h


class BaselineUNet:
    """BaselineUNetImpl(in_channels, init_features, max_depth) on MI355X.

    Extra keyword-only arguments size the device workspace (the reference allocates per call)."""

    MODEL = MODEL_BASELINE

    def __init__(self, in_channels=3, init_features=64, max_depth=10.0, *, batch, height, width, device=0):
        self.lib = _abi.load()
        self.device = torch.device("cuda", device)
        self.in_channels, self.init_features, self.max_depth = in_channels, init_features, max_depth
        self.batch, self.height, self.width = batch, height, width
        desc = _abi.UnetDesc(in_channels, init_features, max_depth, batch, height, width)
        h = C.c_void_p()
        check(self.lib.cad_unet_create_model(C.byref(desc), self.MODEL, device, C.byref(h)), "cad_unet_create_model")
        self.h = h
        self._param_info = [self._info(0, i) for i in range(self.lib.cad_unet_num_params(h))]
        self._buffer_info = [self._info(1, i) for i in range(self.lib.cad_unet_num_buffers(h))]
        n = C.c_int64()
        check(self.lib.cad_unet_flat(h, None, None, C.byref(n)), "cad_unet_flat")
        self.n_flat = n.value
        # flat slabs owned by torch so torch.distributed (RCCL) can all-reduce them in place
        self.flat_params = torch.zeros(self.n_flat, dtype=torch.float32, device=self.device)
        self.flat_grads = torch.zeros(self.n_flat, dtype=torch.float32, device=self.device)
        check(self.lib.cad_unet_use_external_slabs(h, _ptr(self.flat_params), _ptr(self.flat_grads)),
              "cad_unet_use_external_slabs")
        self.num_stages = self.lib.cad_unet_num_stages(h)
        self.stage_ranges = []
        for s in range(self.num_stages):
            off, cnt = C.c_int64(), C.c_int64()
            check(self.lib.cad_unet_stage_grad_range(h, s, C.byref(off), C.byref(cnt)), "stage range")
            self.stage_ranges.append((off.value, cnt.value))
        self.training = True
        self._out = None

    def _info(self, kind, idx):
        name = C.c_char_p()
        nd = C.c_int()
        shape = (C.c_int64 * 4)()
        check(self.lib.cad_unet_tensor_info(self.h, kind, idx, C.byref(name), C.byref(nd), shape), "tensor_info")
        return name.value.decode(), tuple(shape[i] for i in range(nd.value))

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            self.lib.cad_unet_destroy(h)
            self.h = None

    # ---- torch::nn::Module surface used by the trainer ----
    def train(self, mode=True):
        self.training = bool(mode)
        check(self.lib.cad_unet_train(self.h, int(mode)), "cad_unet_train")
        return self

    def eval(self):
        return self.train(False)

    def count_parameters(self) -> int:
        return int(self.lib.cad_unet_count_parameters(self.h))

    def _get(self, kind, idx, shape):
        out = np.empty(int(np.prod(shape)) if shape else 1, np.float32)
        check(self.lib.cad_unet_get_tensor(self.h, kind, idx, out.ctypes.data_as(_abi.FP), out.size), "get_tensor")
        return torch.from_numpy(out.reshape(shape))

    def named_parameters(self):
        torch.cuda.synchronize(self.device)
        return OrderedDict((n, self._get(0, i, s)) for i, (n, s) in enumerate(self._param_info))

    def named_buffers(self):
        torch.cuda.synchronize(self.device)
        return OrderedDict((n, self._get(1, i, s)) for i, (n, s) in enumerate(self._buffer_info))

    def state_dict(self):
        d = self.named_parameters()
        d.update(self.named_buffers())
        return d

    def load_state_dict(self, state, strict=True):
        torch.cuda.synchronize(self.device)
        names = {n: (0, i, s) for i, (n, s) in enumerate(self._param_info)}
        names.update({n: (1, i, s) for i, (n, s) in enumerate(self._buffer_info)})
        missing = [n for n in names if n not in state]
        if strict and missing:
            raise KeyError(f"missing keys: {missing[:5]}")
        for n, (kind, i, s) in names.items():
            if n not in state:
                continue
            v = np.ascontiguousarray(torch.as_tensor(state[n]).detach().cpu().float().numpy())
            assert tuple(v.shape) == tuple(s), f"{n}: shape {v.shape} != {s}"
            check(self.lib.cad_unet_set_tensor(self.h, kind, i, v.ctypes.data_as(_abi.FP), v.size), f"set {n}")

    def grads(self):
        torch.cuda.synchronize(self.device)
        out = OrderedDict()
        for i, (n, s) in enumerate(self._param_info):
            g = np.empty(int(np.prod(s)), np.float32)
            check(self.lib.cad_unet_get_grad(self.h, i, g.ctypes.data_as(_abi.FP), g.size), "get_grad")
            out[n] = torch.from_numpy(g.reshape(s))
        return out

    # ---- forward / backward ----
    @property
    def conditioned(self) -> bool:
        return self.MODEL != MODEL_BASELINE

    def forward(self, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        B, Cc, H, W = x.shape
        assert Cc == self.in_channels and H == self.height and W == self.width, "input shape mismatch"
        if out is None:
            out = torch.empty((B, 1, H, W), dtype=torch.float32, device=self.device)
        check(self.lib.cad_unet_forward(self.h, _ptr(x), _ptr(out), B, _stream(self.device)), "cad_unet_forward")
        return out

    def forward_cam(self, x: torch.Tensor, intrinsics: torch.Tensor, out: torch.Tensor | None = None):
        """forward(x, camera_intrinsics (B,4) [fx, fy, cx, cy]) of the camera-conditioned models."""
        B, Cc, H, W = x.shape
        assert Cc == self.in_channels and H == self.height and W == self.width, "input shape mismatch"
        assert tuple(intrinsics.shape) == (B, 4), "intrinsics must be (B, 4) [fx, fy, cx, cy]"
        if out is None:
            out = torch.empty((B, 1, H, W), dtype=torch.float32, device=self.device)
        check(self.lib.cad_unet_forward_cam(self.h, _ptr(x), _ptr(intrinsics.contiguous()), _ptr(out), B,
                                            _stream(self.device)), "cad_unet_forward_cam")
        return out

    def __call__(self, x, *args, **kw):
        return self.forward_cam(x, *args, **kw) if self.conditioned else self.forward(x, *args, **kw)

    def backward(self, ddepth: torch.Tensor, on_stage=None):
        """Backward of the last train-mode forward. on_stage(stage, offset, count) is called after
        each stage is enqueued (gradients of flat_grads[offset:offset+count] are then final on the
        stream) — the hook the data-parallel trainer uses to overlap RCCL all-reduce."""
        st = _stream(self.device)
        if on_stage is None:
            check(self.lib.cad_unet_backward(self.h, _ptr(ddepth), st), "cad_unet_backward")
            return
        for s in range(self.num_stages):
            check(self.lib.cad_unet_backward_stage(self.h, s, _ptr(ddepth), st), f"backward stage {s}")
            on_stage(s, *self.stage_ranges[s])

    def debug_buffer(self, name: str) -> torch.Tensor:
        """Host copy of an internal NHWC buffer (flat) — debugging / layer-level parity only."""
        n = self.lib.cad_unet_debug_buffer(self.h, name.encode(), None, 0)
        if n < 0:
            raise KeyError(name)
        out = np.empty(n, np.float32)
        assert self.lib.cad_unet_debug_buffer(self.h, name.encode(), out.ctypes.data_as(_abi.FP), n) == n
        return torch.from_numpy(out)

    def num_batches_tracked(self) -> int:
        return int(self.lib.cad_unet_num_batches_tracked(self.h))

    def last_grad_norm(self) -> float:
        v = C.c_float()
        check(self.lib.cad_unet_last_grad_norm(self.h, C.byref(v), _stream(self.device)), "last_grad_norm")
        return float(v.value)


def save(model: BaselineUNet, path: str):
    """torch::save(model_, path) (tensorboard_trainer_enhanced.h:656-662): the TorchScript archive
    LibTorch writes for the module, readable by the reference's torch::load (cad_unet_save_torch)."""
    check(model.lib.cad_unet_save_torch(model.h, str(path).encode()), "cad_unet_save_torch")


def load(model: BaselineUNet, path: str):
    """torch::load(model, path): parameters, BatchNorm buffers and num_batches_tracked from a
    torch::save archive (the reference's or ours); every model tensor must be present with its shape."""
    torch.cuda.synchronize(model.device)
    check(model.lib.cad_unet_load_torch(model.h, str(path).encode()), "cad_unet_load_torch")


class IntrinsicsConditionedUNet(BaselineUNet):
    """IntrinsicsConditionedUNetImpl(in_channels, init_features, camera_dim=4, max_depth) on MI355X:
    a FiLMLayerImpl(4, C) after the first BN-ReLU of every DoubleConv, fed the normalised (B,4)
    intrinsics (intrinsics_unet.h:137-270).  forward(x, intrinsics) takes [fx, fy, cx, cy]."""

    MODEL = MODEL_INTRINSICS_FILM

    def __init__(self, in_channels=3, init_features=64, camera_dim=4, max_depth=10.0, *, batch, height, width,
                 device=0):
        assert camera_dim == 4, "camera_dim 4 ([fx, fy, cx, cy]) is the configuration on the hot path"
        super().__init__(in_channels, init_features, max_depth, batch=batch, height=height, width=width,
                         device=device)

    def forward(self, x, intrinsics, out=None):   # noqa: D401 (reference signature)
        return self.forward_cam(x, intrinsics, out)


class RayConditionedUNet(IntrinsicsConditionedUNet):
    """Config-3 model (SURVEY §8 "Recommended config-3 model"): enc1 = RayEnhancedConv(3, f, 4,
    use_rays=true) fed cat(rgb, per-pixel rays from the intrinsics), FiLM blocks after."""

    MODEL = MODEL_RAY_FILM


def camera_from_K(K: torch.Tensor) -> torch.Tensor:
    """(B,3,3) intrinsics -> (B,4) [fx, fy, cx, cy] on device."""
    B = K.shape[0]
    lib = _abi.load()
    out = torch.empty((B, 4), dtype=torch.float32, device=K.device)
    check(lib.cad_camera_from_K(_ptr(K.reshape(B, 9).contiguous()), B, _ptr(out), _stream(K.device)), "camera_from_K")
    return out


def clip_grad_norm_(model: BaselineUNet, max_norm: float, prescale: float = 1.0):
    """torch::nn::utils::clip_grad_norm_ over all parameters (device-resident total norm)."""
    check(model.lib.cad_clip_grad_norm(model.h, float(max_norm), float(prescale), _stream(model.device)), "clip")


class Adam:
    """torch::optim::Adam(params, AdamOptions(lr).betas(b).eps(eps).weight_decay(wd)) — coupled L2."""

    def __init__(self, model: BaselineUNet, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        self.model = model
        self.lib = model.lib
        o = _abi.AdamOpts(lr, betas[0], betas[1], eps, weight_decay)
        h = C.c_void_p()
        check(self.lib.cad_adam_create(model.h, C.byref(o), C.byref(h)), "cad_adam_create")
        self.h = h

    def step(self):
        check(self.lib.cad_adam_step(self.h, _stream(self.model.device)), "cad_adam_step")

    def zero_grad(self):
        """No-op: every backward overwrites the whole gradient slab (set_to_none semantics)."""

    def set_lr(self, lr):
        check(self.lib.cad_adam_set_lr(self.h, float(lr)), "set_lr")

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            self.lib.cad_adam_destroy(h)
            self.h = None


class CombinedDepthLoss:
    """CombinedDepthLoss(si_weight, grad_weight, smooth_weight, reproj_weight) with its backward
    (depth_loss.h:366-479).  forward_with_intrinsics / forward take the reference's optional
    valid_mask (bool or uint8 device tensor (B,1,H,W)); it replaces gt > 1e-6 in the SI and
    reprojection terms, the gradient-matching term ignores it (depth_loss.h:137)."""

    def __init__(self, si_weight=1.0, grad_weight=0.1, smooth_weight=0.001, reproj_weight=0.01, *, batch, height,
                 width, device=0):
        self.lib = _abi.load()
        self.device = torch.device("cuda", device)
        self.weights = (si_weight, grad_weight, smooth_weight, reproj_weight)
        self.batch, self.height, self.width = batch, height, width
        self.h = self._create(reproj_weight)
        self.h_noreproj = None   # forward() (no reprojection term), created on first use

    def _create(self, reproj_weight):
        h = C.c_void_p()
        si, gr, sm, _ = self.weights
        check(self.lib.cad_loss_create(si, gr, sm, reproj_weight, self.batch, self.height, self.width,
                                       self.device.index or 0, C.byref(h)), "cad_loss_create")
        return h

    def __del__(self):
        for attr in ("h", "h_noreproj"):
            h = getattr(self, attr, None)
            if h is not None and h.value:
                self.lib.cad_loss_destroy(h)
                setattr(self, attr, None)

    def _run(self, h, pred, gt, image, intrinsics, valid_mask, loss5, dpred):
        B = pred.shape[0]
        assert pred.shape[2] == self.height and pred.shape[3] == self.width
        K = intrinsics.reshape(B, 3, 3).contiguous()
        if loss5 is None:
            loss5 = torch.empty(5, dtype=torch.float32, device=self.device)
        if dpred is None:
            dpred = torch.empty_like(pred)
        m = None
        if valid_mask is not None:
            assert valid_mask.numel() == pred.numel(), "valid_mask must be (B,1,H,W)"
            mt = valid_mask.reshape(pred.shape).to(torch.uint8).contiguous()
            m = C.c_void_p(mt.data_ptr())
        check(self.lib.cad_loss_forward_backward_masked(h, _ptr(pred), _ptr(gt), _ptr(image), _ptr(K), m, B,
                                                        _ptr(loss5), _ptr(dpred), _stream(self.device)),
              "cad_loss_forward_backward")
        return loss5, dpred

    def forward_with_intrinsics(self, pred, gt, image, intrinsics, valid_mask=None, loss5=None, dpred=None):
        """forwardWithIntrinsics + backward. Returns (loss5, dpred): loss5 = device tensor
        [total, si, grad, smooth, reproj]; dpred = dL/dpred (B,1,H,W)."""
        return self._run(self.h, pred, gt, image, intrinsics, valid_mask, loss5, dpred)

    forwardWithIntrinsics = forward_with_intrinsics

    def forward(self, pred, gt, image, valid_mask=None, loss5=None, dpred=None):
        """forward (depth_loss.h:390-404): SI + grad + smooth, no reprojection term (the kernels still
        take intrinsics for their pixel grid; identity K is passed)."""
        if self.h_noreproj is None:
            self.h_noreproj = self._create(0.0)
        B = pred.shape[0]
        K = torch.eye(3, dtype=torch.float32, device=self.device).expand(B, 3, 3).contiguous()
        return self._run(self.h_noreproj, pred, gt, image, K, valid_mask, loss5, dpred)

    def get_components_with_intrinsics(self, pred, gt, image, intrinsics, valid_mask=None):
        """getComponentsWithIntrinsics: the four terms (host floats); scratch outputs of its own, so a
        caller's loss5 / dL/dpred are left as they were."""
        loss5, _ = self.forward_with_intrinsics(pred, gt, image, intrinsics, valid_mask)
        v = loss5.cpu().tolist()
        return {"si_loss": v[1], "grad_loss": v[2], "smooth_loss": v[3], "reproj_loss": v[4]}

    getComponentsWithIntrinsics = get_components_with_intrinsics

    def get_components(self, pred, gt, image, valid_mask=None):
        loss5, _ = self.forward(pred, gt, image, valid_mask)
        v = loss5.cpu().tolist()
        return {"si_loss": v[1], "grad_loss": v[2], "smooth_loss": v[3]}

    getComponents = get_components


def depth_metrics(pred: torch.Tensor, gt: torch.Tensor) -> dict:
    """computeDepthMetrics (enhanced.h:400-439) per sample, averaged over the batch."""
    lib = _abi.load()
    B, _, H, W = pred.shape
    out = (C.c_float * 7)()
    check(lib.cad_depth_metrics(_ptr(pred), _ptr(gt), B, H, W, out, _stream(pred.device)), "cad_depth_metrics")
    keys = ["abs_rel", "sq_rel", "rmse", "rmse_log", "a1", "a2", "a3"]
    return {k: float(out[i]) for i, k in enumerate(keys)}


def ray_directions(K: torch.Tensor, height: int, width: int) -> torch.Tensor:
    """RayDirectionComputer::computeRayDirections for a batch of K (B,3,3) -> (B,3,H,W)."""
    lib = _abi.load()
    B = K.shape[0]
    out = torch.empty((B, 3, height, width), dtype=torch.float32, device=K.device)
    check(lib.cad_ray_directions(_ptr(K.contiguous()), B, height, width, _ptr(out), _stream(K.device)), "rays")
    return out


class GradBucketer:
    """Decoder-first gradient buckets for the data-parallel all-reduce.

    Backward stages finish in decreasing flat-slab offset order (head, dec1..dec4, bottleneck,
    enc4..enc1), so consecutive stages form contiguous slices.  A slice is launched (async, RCCL over
    xGMI via torch.distributed) as soon as it holds >= bucket_elems floats or the last stage ends;
    the launch records an event on the current stream, so the collective overlaps the remaining
    backward kernels.  Every element is reduced exactly once (SUM; the 1/world mean is folded into
    clip + Adam)."""

    def __init__(self, flat: torch.Tensor, num_stages: int, bucket_elems: int, process_group=None):
        self.flat, self.num_stages, self.bucket_elems, self.pg = flat, num_stages, bucket_elems, process_group
        self.pending = []
        self.lo = self.hi = None
        self.buckets = []

    def on_stage(self, stage, off, cnt):
        lo, hi = off, off + cnt
        self.lo = lo if self.lo is None else min(self.lo, lo)
        self.hi = hi if self.hi is None else max(self.hi, hi)
        if self.hi - self.lo >= self.bucket_elems or stage == self.num_stages - 1:
            self.flush()

    def flush(self):
        import torch.distributed as dist
        if self.lo is None:
            return
        self.buckets.append((self.lo, self.hi))
        self.pending.append(dist.all_reduce(self.flat[self.lo:self.hi], group=self.pg, async_op=True))
        self.lo = self.hi = None

    def wait(self):
        for w in self.pending:
            w.wait()
        self.pending = []


class Communicator:
    """RCCL communicator of libcad (cad_comm_* in cad.h; C++: cad::distributed::Communicator), the
    data-parallel exchange build/train uses: one rank per GPU, rank 0's 128-byte unique id handed to
    the others out of band (a file, a torch.distributed broadcast_object_list, ...).

    backward_allreduce(model, ddepth) runs the backward with the decoder-first bucketed SUM
    all-reduce issued on the communicator's own stream as each bucket's last stage is enqueued; the
    caller's stream waits for the last one, so clip (prescale 1/world) and Adam see the reduced slab."""

    @staticmethod
    def unique_id() -> bytes:
        lib = _abi.load()
        buf = (C.c_uint8 * 128)()
        check(lib.cad_comm_get_unique_id(buf), "cad_comm_get_unique_id")
        return bytes(buf)

    def __init__(self, uid: bytes, world: int, rank: int, device: int = 0):
        assert len(uid) == 128, "unique id is 128 bytes"
        self.lib = _abi.load()
        self.device = torch.device("cuda", device)
        h = C.c_void_p()
        check(self.lib.cad_comm_create((C.c_uint8 * 128)(*uid), world, rank, device, C.byref(h)), "cad_comm_create")
        self.h = h

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            self.lib.cad_comm_destroy(h)
            self.h = None

    def rank(self) -> int:
        return self.lib.cad_comm_rank(self.h)

    def size(self) -> int:
        return self.lib.cad_comm_size(self.h)

    def set_timing(self, on=True):
        """Time every backward_allreduce from now on (cad_comm_set_timing): exposed exchange time and
        all-reduce span per call, read by stats()."""
        check(self.lib.cad_comm_set_timing(self.h, int(bool(on))), "cad_comm_set_timing")
        return self

    def stats(self) -> dict:
        """Exchange accounting since the last read (cad_comm_stats_read; waits for the recorded events):
        calls, buckets, bytes all-reduced, and over the timed calls the summed exposed time (last
        backward kernel -> compute stream released by the last all-reduce) and all-reduce span."""
        s = _abi.CommStats()
        check(self.lib.cad_comm_stats_read(self.h, C.byref(s)), "cad_comm_stats_read")
        return {"calls": s.calls, "timed_calls": s.timed_calls, "buckets": s.buckets, "bytes": s.bytes,
                "exposed_ms": s.exposed_ms, "span_ms": s.span_ms}

    def allreduce(self, t: torch.Tensor, op="sum"):
        check(self.lib.cad_comm_allreduce(self.h, _ptr(t), t.numel(), {"sum": 0, "max": 1}[op], _stream(self.device)),
              "cad_comm_allreduce")
        return t

    def broadcast_parameters(self, model, root=0):
        """Identical replicas: the flat parameter slab of `model` (any family) from rank `root`."""
        if isinstance(model, BaselineUNet):
            check(self.lib.cad_comm_broadcast_params(model.h, self.h, root, _stream(self.device)), "broadcast_params")
        else:
            check(self.lib.cad_comm_broadcast(self.h, model._flat_p, model.n_flat, root, _stream(self.device)),
                  "cad_comm_broadcast")

    def backward_allreduce(self, model, ddepth: torch.Tensor, bucket_elems=25 << 18):
        """The model's staged backward with the overlapped SUM exchange (cad_unet_backward_allreduce,
        cad_resunet_backward_allreduce, cad_geonet_backward_allreduce)."""
        fn = (self.lib.cad_unet_backward_allreduce if isinstance(model, BaselineUNet)
              else getattr(self.lib, model._PREFIX + "backward_allreduce"))
        check(fn(model.h, self.h, _ptr(ddepth), bucket_elems, _stream(self.device)), "backward_allreduce")


class Trainer:
    """One optimisation step of TensorBoardTrainerEnhanced::trainEpoch (enhanced.h:287-304):
    zero_grad, forward, forwardWithIntrinsics, backward, clip_grad_norm_(max 1.0), Adam.step.

    Data-parallel: with `process_group` set, gradient buckets are all-reduced
    (RCCL over xGMI via torch.distributed) as soon as their backward stage is enqueued, overlapping
    the rest of the backward; the mean (1/world) is folded into clip + Adam.  BN statistics and
    loss masks stay per replica (DDP semantics, no SyncBN).  With `communicator` (a libcad
    Communicator) the same exchange runs inside the library (cad_unet_backward_allreduce), as in
    build/train."""

    def __init__(self, model: BaselineUNet, loss_fn: CombinedDepthLoss, lr=1e-4, weight_decay=1e-5,
                 grad_clip=1.0, use_grad_clip=True, process_group=None, bucket_mb=25.0, communicator=None):
        self.model, self.loss_fn = model, loss_fn
        self.optimizer = Adam(model, lr=lr, weight_decay=weight_decay)
        self.grad_clip = grad_clip if use_grad_clip else float("inf")
        self.pg = process_group
        self.comm = communicator
        self.world = 1
        assert process_group is None or communicator is None, "one gradient exchange"
        if communicator is not None:
            self.world = communicator.size()
        if process_group is not None:
            import torch.distributed as dist
            self.world = dist.get_world_size(process_group)
        self.bucket_elems = int(bucket_mb * (1 << 20) / 4)
        self.pred = None
        self.loss5 = torch.zeros(5, dtype=torch.float32, device=model.device)
        self.timing = False
        self._events = []
        self._xstats = {"calls": 0, "buckets": 0, "bytes": 0}

    def set_exchange_timing(self, on=True):
        """Account the data-parallel exchange of the following steps (exchange_stats())."""
        self.timing = bool(on)
        if self.comm is not None:
            self.comm.set_timing(on)
        return self

    def exchange_stats(self) -> dict:
        """Gradient-exchange accounting since the last read: the communicator's rank count, bytes
        all-reduced, buckets, and the exposed (non-overlapped) exchange time summed over timed steps
        (libcad communicator: cad_comm_stats_read; torch.distributed: CUDA events around the wait)."""
        if self.comm is not None:
            out = self.comm.stats()
            out.update(backend="libcad RCCL communicator", comm_size=self.comm.size())
            return out
        if self.pg is None:
            return {"backend": None, "comm_size": 1, "calls": 0, "timed_calls": 0, "buckets": 0, "bytes": 0,
                    "exposed_ms": 0.0, "span_ms": None}
        import torch.distributed as dist
        torch.cuda.synchronize(self.model.device)
        out = dict(self._xstats, timed_calls=len(self._events),
                   exposed_ms=sum(a.elapsed_time(b) for a, b in self._events), span_ms=None,
                   backend=f"torch.distributed ({dist.get_backend(self.pg)})", comm_size=dist.get_world_size(self.pg))
        self._events = []
        self._xstats = {"calls": 0, "buckets": 0, "bytes": 0}
        return out

    def train_step(self, rgb, gt, K):
        m = self.model
        m.train()
        self.optimizer.zero_grad()
        B = rgb.shape[0]
        if self.pred is None or self.pred.shape[0] != B:
            self.pred = torch.empty((B, 1, m.height, m.width), dtype=torch.float32, device=m.device)
            self.dpred = torch.empty_like(self.pred)
            self.cam4 = torch.empty((B, 4), dtype=torch.float32, device=m.device)
        if m.conditioned:   # camera vector from the batch intrinsics (a15), then the FiLM forward
            check(m.lib.cad_camera_from_K(_ptr(K.reshape(B, 9).contiguous()), B, _ptr(self.cam4),
                                          _stream(m.device)), "camera_from_K")
            m.forward_cam(rgb, self.cam4, out=self.pred)
        else:
            m.forward(rgb, out=self.pred)
        self.loss_fn.forward_with_intrinsics(self.pred, gt, rgb, K, loss5=self.loss5, dpred=self.dpred)
        if self.comm is not None:
            self.comm.backward_allreduce(m, self.dpred, self.bucket_elems)
            clip_grad_norm_(m, self.grad_clip, prescale=1.0 / self.world)
        elif self.world > 1:
            bk = GradBucketer(m.flat_grads, m.num_stages, self.bucket_elems, self.pg)
            m.backward(self.dpred, on_stage=bk.on_stage)
            ev = None
            if self.timing:   # exposed exchange time: after the last backward kernel -> after the wait
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            bk.wait()
            if ev is not None:
                ev[1].record()
                self._events.append(ev)
            self._xstats["calls"] += 1
            self._xstats["buckets"] += len(bk.buckets)
            self._xstats["bytes"] += 4 * sum(hi - lo for lo, hi in bk.buckets)
            clip_grad_norm_(m, self.grad_clip, prescale=1.0 / self.world)
        else:
            m.backward(self.dpred)
            clip_grad_norm_(m, self.grad_clip)
        self.optimizer.step()
        return self.loss5


class ResNetUNet:
    """Config-5 network (BASELINE configs[4]): ResNet-50 encoder + U-Net decoder on MI355X, bf16
    operands (cad_resunet_*; resunet.cpp).  No reference model exists — parity is unpinned and the
    network is checked against the torch fp32 restatement in oracle/resunet_oracle.py.

    Parameter names follow torchvision's ResNet-50 under "encoder." and the U-Net decoder
    ("dec4".."dec0", "out_conv").  train_step() = forward, CombinedDepthLoss, backward,
    clip_grad_norm_, Adam (moments owned by the model)."""

    _PREFIX = "cad_resunet_"

    def _f(self, name):
        return getattr(self.lib, self._PREFIX + name)

    def __init__(self, in_channels=3, max_depth=10.0, *, batch, height, width, device=0, fp8=False):
        self.lib = _abi.load()
        self.device = torch.device("cuda", device)
        self.batch, self.height, self.width, self.max_depth = batch, height, width, max_depth
        desc = _abi.ResUnetDesc(in_channels, batch, height, width, max_depth)
        h = C.c_void_p()
        check(self._f("create")(C.byref(desc), device, C.byref(h)), "cad_resunet_create")
        self._init_handle(h)
        self.set_fp8(fp8)

    def set_fp8(self, on=True):
        """MX-fp8 forward conv-GEMMs (cad_resunet_set_fp8): every eligible forward contraction on OCP
        MXFP8 E4M3 operands (one E8M0 scale per 32 channels); the backward stays on bf16 operands."""
        check(self._f("set_fp8")(self.h, int(bool(on))), "cad_resunet_set_fp8")
        self.fp8 = bool(on)
        return self

    @property
    def fp8_units(self) -> int:
        """number of convolutions whose forward runs on MX-fp8 operands when fp8 is on"""
        return int(self._f("fp8_units")(self.h))

    def _init_handle(self, h):
        self.h = h
        self._param_info = [self._info(0, i) for i in range(self._f("num_tensors")(h, 0))]
        self._buffer_info = [self._info(1, i) for i in range(self._f("num_tensors")(h, 1))]
        p, g, n = C.c_void_p(), C.c_void_p(), C.c_int64()
        check(self._f("flat")(h, C.byref(p), C.byref(g), C.byref(n)), "flat")
        self.n_flat = n.value
        self._flat_p = p.value
        self._flat_g = g.value
        self.num_stages = self._f("num_stages")(h)
        self.stage_ranges = []
        for st in range(self.num_stages):
            off, cnt = C.c_int64(), C.c_int64()
            check(self._f("stage_grad_range")(h, st, C.byref(off), C.byref(cnt)), "stage range")
            self.stage_ranges.append((off.value, cnt.value))
        self.training = True

    def _info(self, kind, idx):
        name, nd, shape = C.c_char_p(), C.c_int(), (C.c_int64 * 4)()
        check(self._f("tensor_info")(self.h, kind, idx, C.byref(name), C.byref(nd), shape), "tensor_info")
        return name.value.decode(), tuple(shape[i] for i in range(nd.value))

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            self._f("destroy")(h)
            self.h = None

    def train(self, mode=True):
        self.training = bool(mode)
        check(self._f("train")(self.h, int(mode)), "cad_resunet_train")
        return self

    def eval(self):
        return self.train(False)

    def count_parameters(self) -> int:
        return int(self._f("count_parameters")(self.h))

    def _get(self, kind, idx, shape):
        out = np.empty(int(np.prod(shape)) if shape else 1, np.float32)
        check(self._f("get_tensor")(self.h, kind, idx, out.ctypes.data_as(_abi.FP), out.size), "get_tensor")
        return torch.from_numpy(out.reshape(shape))

    def named_parameters(self):
        torch.cuda.synchronize(self.device)
        return OrderedDict((n, self._get(0, i, s)) for i, (n, s) in enumerate(self._param_info))

    def named_buffers(self):
        torch.cuda.synchronize(self.device)
        return OrderedDict((n, self._get(1, i, s)) for i, (n, s) in enumerate(self._buffer_info))

    def state_dict(self):
        d = self.named_parameters()
        d.update(self.named_buffers())
        return d

    def load_state_dict(self, state, strict=True):
        torch.cuda.synchronize(self.device)
        names = {n: (0, i, s) for i, (n, s) in enumerate(self._param_info)}
        names.update({n: (1, i, s) for i, (n, s) in enumerate(self._buffer_info)})
        missing = [n for n in names if n not in state]
        if strict and missing:
            raise KeyError(f"missing keys: {missing[:5]}")
        for n, (kind, i, s) in names.items():
            if n not in state:
                continue
            v = np.ascontiguousarray(torch.as_tensor(state[n]).detach().cpu().float().numpy())
            assert tuple(v.shape) == tuple(s), f"{n}: shape {v.shape} != {s}"
            check(self._f("set_tensor")(self.h, kind, i, v.ctypes.data_as(_abi.FP), v.size), f"set {n}")

    def grads(self):
        torch.cuda.synchronize(self.device)
        out = OrderedDict()
        for i, (n, s) in enumerate(self._param_info):
            g = np.empty(int(np.prod(s)), np.float32)
            check(self._f("get_grad")(self.h, i, g.ctypes.data_as(_abi.FP), g.size), "get_grad")
            out[n] = torch.from_numpy(g.reshape(s))
        return out

    def flat_grads_ptr(self) -> int:
        """Device address of the flat gradient slab (n_flat floats): the data-parallel all-reduce buffer."""
        return self._flat_g

    def debug_buffer(self, name: str) -> torch.Tensor:
        """Test hook: a buffer of the last train-mode forward as fp32 NHWC rows (cad_resunet_debug_buffer:
        "y:<conv>" stored pre-BN outputs, "scale:<bn>" / "shift:<bn>" BN-apply coefficients, "out:<block>"
        block outputs, "cat:dec<l>" a decoder's bf16 input [skip, up])."""
        n = int(self._f("debug_buffer")(self.h, name.encode(), None, 0))
        if n < 0:
            raise KeyError(name)
        out = np.empty(n, np.float32)
        check(0 if self._f("debug_buffer")(self.h, name.encode(), out.ctypes.data_as(_abi.FP), n) == n else 1, name)
        if name.startswith(("amax", "sidx")):
            out = out.view(np.int32)
        return torch.from_numpy(out)

    def forward(self, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        B, Cc, H, W = x.shape
        assert Cc == 3 and H == self.height and W == self.width and B <= self.batch, "input shape mismatch"
        if out is None:
            out = torch.empty((B, 1, H, W), dtype=torch.float32, device=self.device)
        check(self._f("forward")(self.h, _ptr(x), _ptr(out), B, _stream(self.device)), "cad_resunet_forward")
        return out

    __call__ = forward

    @property
    def flat_grads(self) -> torch.Tensor:
        """A torch view of the flat gradient slab (the data-parallel all-reduce buffer)."""
        return _flat_view(self._flat_g, self.n_flat, self.device)

    @property
    def flat_params(self) -> torch.Tensor:
        return _flat_view(self._flat_p, self.n_flat, self.device)

    def backward(self, ddepth: torch.Tensor, on_stage=None):
        """Backward of the last train-mode forward; on_stage(stage, offset, count) after each stage is
        enqueued (its gradients flat_grads[offset:offset+count] are then final on the stream)."""
        st = _stream(self.device)
        if on_stage is None:
            check(self._f("backward")(self.h, _ptr(ddepth), st), self._PREFIX + "backward")
            return
        for s in range(self.num_stages):
            check(self._f("backward_stage")(self.h, s, _ptr(ddepth), st), f"backward stage {s}")
            on_stage(s, *self.stage_ranges[s])

    def _exchange_backward(self, dpred, process_group, communicator, bucket_mb):
        """backward + the data-parallel SUM exchange of the gradient slab; returns the world size."""
        if communicator is not None:
            communicator.backward_allreduce(self, dpred, int(bucket_mb * (1 << 20) / 4))
            return communicator.size()
        if process_group is not None:
            import torch.distributed as dist
            bk = GradBucketer(self.flat_grads, self.num_stages, int(bucket_mb * (1 << 20) / 4), process_group)
            self.backward(dpred, on_stage=bk.on_stage)
            acct = getattr(self, "_xacct", None)   # exchange_accounting(): events around the wait
            if acct is not None:
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            bk.wait()
            if acct is not None:
                ev[1].record()
                acct["events"].append(ev)
                acct["calls"] += 1
                acct["buckets"] += len(bk.buckets)
                acct["bytes"] += 4 * sum(hi - lo for lo, hi in bk.buckets)
                acct["pg"] = process_group
            return dist.get_world_size(process_group)
        self.backward(dpred)
        return 1

    def exchange_accounting(self, on=True):
        """torch.distributed exchange of train_step(process_group=...): count buckets / bytes and time
        the exposed wait from now on (exchange_stats()); a libcad Communicator accounts on its own
        (Communicator.set_timing / stats)."""
        self._xacct = {"events": [], "calls": 0, "buckets": 0, "bytes": 0, "pg": None} if on else None
        return self

    def exchange_stats(self) -> dict:
        import torch.distributed as dist
        a = getattr(self, "_xacct", None) or {"events": [], "calls": 0, "buckets": 0, "bytes": 0, "pg": None}
        torch.cuda.synchronize(self.device)
        out = {"calls": a["calls"], "timed_calls": len(a["events"]), "buckets": a["buckets"], "bytes": a["bytes"],
               "exposed_ms": sum(x.elapsed_time(y) for x, y in a["events"]), "span_ms": None,
               "backend": f"torch.distributed ({dist.get_backend(a['pg'])})" if a["pg"] is not None else None,
               "comm_size": dist.get_world_size(a["pg"]) if a["pg"] is not None else 1}
        if getattr(self, "_xacct", None) is not None:
            self.exchange_accounting(True)
        return out

    def clip_grad_norm_(self, max_norm: float, prescale: float = 1.0):
        check(self._f("clip_grad_norm")(self.h, float(max_norm), float(prescale), _stream(self.device)), "clip")

    def last_grad_norm(self) -> float:
        v = C.c_float()
        check(self._f("last_grad_norm")(self.h, C.byref(v), _stream(self.device)), "last_grad_norm")
        return float(v.value)

    def adam_step(self, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-5):
        check(self._f("adam_step")(self.h, lr, betas[0], betas[1], eps, weight_decay, _stream(self.device)),
              "adam_step")

    def train_step(self, loss_fn: "CombinedDepthLoss", rgb, gt, K, lr=1e-4, weight_decay=1e-5, grad_clip=1.0,
                   pred=None, dpred=None, loss5=None, process_group=None, communicator=None, bucket_mb=25.0):
        """One optimisation step (enhanced.h:287-304 sequence).  Data-parallel (process_group over
        torch.distributed, or a libcad Communicator): decoder-first gradient buckets SUM-all-reduced
        while the rest of the backward runs, clipped as the mean."""
        pred = self.forward(rgb, out=pred)
        loss5, dpred = loss_fn.forward_with_intrinsics(pred, gt, rgb, K, loss5=loss5, dpred=dpred)
        world = self._exchange_backward(dpred, process_group, communicator, bucket_mb)
        self.clip_grad_norm_(grad_clip if grad_clip else float("inf"), 1.0 / world)
        self.adam_step(lr=lr, weight_decay=weight_decay)
        return loss5, pred


class GeometryAwareNetwork(ResNetUNet):
    """GeometryAwareNetworkImpl(in_channels, init_features, camera_dim, max_depth, use_pcl, use_attention)
    (src/models/geometry_aware_network.h:201-347) on MI355X (cad_geonet_*; geonet.cpp): RayEnhancedConv
    encoder with CBAM, ConvTranspose + PerspectiveCorrectionLayer + CBAM decoder, six levels.
    forward(rgb, ray_directions, camera_intrinsics (B,4)) as the reference; parameter / buffer names
    are its named_parameters() / named_buffers().  Arithmetic: the process GEMM engine (default S3,
    fp32-accurate).  train_step(): forward, CombinedDepthLoss, backward, clip_grad_norm_, Adam."""

    _PREFIX = "cad_geonet_"
    _VARIANT = 0

    def __init__(self, in_channels=3, init_features=64, camera_dim=4, max_depth=10.0, use_pcl=True,
                 use_attention=True, *, batch, height, width, device=0):
        self.lib = _abi.load()
        self.device = torch.device("cuda", device)
        self.batch, self.height, self.width, self.max_depth = batch, height, width, max_depth
        desc = _abi.GeoNetDesc(self._VARIANT, in_channels, init_features, camera_dim, max_depth, int(use_pcl),
                               int(use_attention), batch, height, width)
        h = C.c_void_p()
        check(self._f("create")(C.byref(desc), device, C.byref(h)), "cad_geonet_create")
        self._init_handle(h)

    def forward(self, rgb, ray_directions, camera_intrinsics, out=None):
        B, Cc, H, W = rgb.shape
        assert Cc == 3 and H == self.height and W == self.width and B <= self.batch, "input shape mismatch"
        assert tuple(ray_directions.shape) == (B, 3, H, W), "ray_directions must be (B, 3, H, W)"
        assert tuple(camera_intrinsics.shape) == (B, 4), "camera_intrinsics must be (B, 4) [fx, fy, cx, cy]"
        rgb, rays, cam = (t.contiguous().float() for t in (rgb, ray_directions, camera_intrinsics))
        if out is None:
            out = torch.empty((B, 1, H, W), dtype=torch.float32, device=self.device)
        check(self._f("forward")(self.h, _ptr(rgb), _ptr(rays), _ptr(cam), _ptr(out), B, _stream(self.device)),
              "cad_geonet_forward")
        return out

    __call__ = forward

    def num_batches_tracked(self, film=False) -> int:
        return int(self._f("num_batches_tracked")(self.h, int(film)))

    def debug_buffer(self, name: str) -> torch.Tensor:
        """Test hook: a buffer of the last step as NHWC rows ("cat<l>", "dcat<l>", "x<l>", "u<l>", "z<l>",
        the pre-BN conv outputs "y1<e|d><l>", "y2<e|d><l>"; int32: the CBAM decisions "amax<e|d><l>",
        "sidx<e|d><l>")."""
        return ResNetUNet.debug_buffer(self, name)
        if n < 0:
            raise KeyError(name)
        out = np.empty(n, np.float32)
        check(0 if self._f("debug_buffer")(self.h, name.encode(), out.ctypes.data_as(_abi.FP), n) == n else 1, name)
        if name.startswith(("amax", "sidx")):
            out = out.view(np.int32)
        return torch.from_numpy(out)

    def train_step(self, loss_fn: "CombinedDepthLoss", rgb, gt, K, lr=1e-4, weight_decay=1e-5, grad_clip=1.0,
                   rays=None, pred=None, dpred=None, loss5=None, process_group=None, communicator=None,
                   bucket_mb=25.0):
        """One optimisation step (enhanced.h:287-304 sequence) fed the loader's batch: rays default to
        RayDirectionComputer's from K (a18), intrinsics = [K00, K11, K02, K12] (a15).  Data-parallel
        exchange as ResNetUNet.train_step."""
        if rays is None:
            rays = ray_directions(K, rgb.shape[2], rgb.shape[3])
        pred = self.forward(rgb, rays, camera_from_K(K), out=pred)
        loss5, dpred = loss_fn.forward_with_intrinsics(pred, gt, rgb, K, loss5=loss5, dpred=dpred)
        world = self._exchange_backward(dpred, process_group, communicator, bucket_mb)
        self.clip_grad_norm_(grad_clip if grad_clip else float("inf"), 1.0 / world)
        self.adam_step(lr=lr, weight_decay=weight_decay)
        return loss5, pred


class LightweightGeometryNetwork(GeometryAwareNetwork):
    """LightweightGeometryNetworkImpl(in_channels, init_features=32, camera_dim, max_depth)
    (geometry_aware_network.h:355-440): five levels, PCL and CBAM always on."""

    _VARIANT = 1

    def __init__(self, in_channels=3, init_features=32, camera_dim=4, max_depth=10.0, *, batch, height, width,
                 device=0):
        super().__init__(in_channels, init_features, camera_dim, max_depth, True, True, batch=batch, height=height,
                         width=width, device=device)


def _flat_view(addr: int, n: int, device) -> torch.Tensor:
    """A torch view of a libcad-owned device slab (for torch.distributed collectives)."""
    class _A:
        __cuda_array_interface__ = {"shape": (n,), "typestr": "<f4", "data": (addr, False), "version": 3}
    return torch.as_tensor(_A(), device=device)

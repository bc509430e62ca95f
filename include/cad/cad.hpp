// cad.hpp — header-only C++ drop-in for the reference's hot-path classes, over the C ABI (cad.h).
//
// Same namespace, class names and argument meaning as the reference; device tensors (cad::DeviceTensor,
// NCHW fp32) replace torch::Tensor at the API edge.  Errors throw std::runtime_error, like the
// reference's LibTorch / std::runtime_error paths (train_main.cpp:503-506 prints "Error: <what>").
//
//   camera_aware_depth::BaselineUNetImpl   src/models/baseline_unet.h:122-208
//   camera_aware_depth::CombinedDepthLoss  src/loss/depth_loss.h:366-479
//   camera_aware_depth::optim::Adam        torch::optim::Adam (tensorboard_trainer_enhanced.h:97-101)
//   camera_aware_depth::clip_grad_norm_    torch::nn::utils::clip_grad_norm_ (enhanced.h:300-302)
#ifndef CAD_CAD_HPP
#define CAD_CAD_HPP

#include <array>
#include <cstdint>
#include <map>
#include <memory>
#include <numeric>
#include <optional>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "cad.h"

namespace cad {

inline void check(cad_status s, const char* what) {
    if (s != CAD_OK) throw std::runtime_error(std::string(what) + ": " + cad_last_error());
}

// owning (or borrowed) device tensor view, NCHW fp32
struct DeviceTensor {
    float* data = nullptr;
    std::vector<int64_t> shape;
    int device = 0;
    std::shared_ptr<void> owner;

    int dim() const { return (int)shape.size(); }
    int64_t size(int d) const { return shape.at(d < 0 ? d + dim() : d); }
    int64_t numel() const {
        return std::accumulate(shape.begin(), shape.end(), int64_t(1), std::multiplies<int64_t>());
    }
    static DeviceTensor empty(std::vector<int64_t> shape, int device = 0) {
        DeviceTensor t;
        t.shape = std::move(shape);
        t.device = device;
        void* p = nullptr;
        check(cad_malloc(device, t.numel() * (int64_t)sizeof(float), &p), "cad_malloc");
        t.data = static_cast<float*>(p);
        t.owner = std::shared_ptr<void>(p, [](void* q) { cad_free(q); });
        return t;
    }
    static DeviceTensor from_host(const float* host, std::vector<int64_t> shape, int device = 0) {
        DeviceTensor t = empty(std::move(shape), device);
        check(cad_memcpy(t.data, host, t.numel() * (int64_t)sizeof(float), 0, nullptr), "cad_memcpy h2d");
        return t;
    }
    std::vector<float> to_host() const {
        std::vector<float> h((size_t)numel());
        check(cad_memcpy(h.data(), data, numel() * (int64_t)sizeof(float), 1, nullptr), "cad_memcpy d2h");
        return h;
    }
};

// device bool mask (B,1,H,W) as bytes, nonzero = valid: the reference's optional valid_mask tensor
struct DeviceMask {
    uint8_t* data = nullptr;
    std::vector<int64_t> shape;
    int device = 0;
    std::shared_ptr<void> owner;
    int64_t numel() const {
        return std::accumulate(shape.begin(), shape.end(), int64_t(1), std::multiplies<int64_t>());
    }
    static DeviceMask from_host(const uint8_t* host, std::vector<int64_t> shape, int device = 0) {
        DeviceMask m;
        m.shape = std::move(shape);
        m.device = device;
        void* p = nullptr;
        check(cad_malloc(device, m.numel(), &p), "cad_malloc");
        m.data = static_cast<uint8_t*>(p);
        m.owner = std::shared_ptr<void>(p, [](void* q) { cad_free(q); });
        check(cad_memcpy(m.data, host, m.numel(), 0, nullptr), "cad_memcpy h2d");
        return m;
    }
};

struct Workspace {   // device workspace sizing (the reference allocates per call)
    int batch = 1, height = 480, width = 640, device = 0;
};

}  // namespace cad

namespace camera_aware_depth {

using cad::DeviceTensor;

struct NamedTensor {
    std::string name;
    std::vector<int64_t> shape;
    std::vector<float> value;   // reference layout (OIHW conv, (Cin,Cout,2,2) ConvTranspose)
};

class BaselineUNetImpl {
public:
    explicit BaselineUNetImpl(int in_channels = 3, int init_features = 64, float max_depth_value = 10.0f,
                              cad::Workspace ws = {})
        : BaselineUNetImpl(CAD_MODEL_BASELINE, in_channels, init_features, max_depth_value, ws) {}
    ~BaselineUNetImpl() { cad_unet_destroy(h_); }
    BaselineUNetImpl(const BaselineUNetImpl&) = delete;
    BaselineUNetImpl& operator=(const BaselineUNetImpl&) = delete;

    // forward(x): (B,3,H,W) in [0,1] -> depth (B,1,H,W) in (0, max_depth)   (baseline_unet.h:174-195)
    DeviceTensor forward(const DeviceTensor& x, void* stream = nullptr) {
        if (x.dim() != 4 || x.size(1) != 3) throw std::runtime_error("forward: expected (B,3,H,W)");
        DeviceTensor out = DeviceTensor::empty({x.size(0), 1, x.size(2), x.size(3)}, ws_.device);
        cad::check(cad_unet_forward(h_, x.data, out.data, (int)x.size(0), stream), "forward");
        return out;
    }
    DeviceTensor operator()(const DeviceTensor& x) { return forward(x); }
    void forward_into(const DeviceTensor& x, DeviceTensor& out, void* stream = nullptr) {
        cad::check(cad_unet_forward(h_, x.data, out.data, (int)x.size(0), stream), "forward");
    }
    // loss.backward() through the network (enhanced.h:297), given dL/ddepth
    void backward(const DeviceTensor& ddepth, void* stream = nullptr) {
        cad::check(cad_unet_backward(h_, ddepth.data, stream), "backward");
    }
    int64_t count_parameters() const { return cad_unet_count_parameters(h_); }
    void train(bool on = true) { cad::check(cad_unet_train(h_, on ? 1 : 0), "train"); }
    void eval() { train(false); }

    std::vector<NamedTensor> named_parameters() const { return fetch(0); }
    std::vector<NamedTensor> named_buffers() const { return fetch(1); }
    std::vector<NamedTensor> named_grads() const {
        auto v = fetch(0);
        for (size_t i = 0; i < v.size(); ++i)
            cad::check(cad_unet_get_grad(h_, (int)i, v[i].value.data(), (int64_t)v[i].value.size()), "get_grad");
        return v;
    }
    // load by name (parameters and buffers); returns the number of tensors loaded
    int load(const std::vector<NamedTensor>& ts) {
        int n = 0;
        for (int kind = 0; kind < 2; ++kind) {
            const int cnt = kind == 0 ? cad_unet_num_params(h_) : cad_unet_num_buffers(h_);
            for (int i = 0; i < cnt; ++i) {
                const char* name;
                cad::check(cad_unet_tensor_info(h_, kind, i, &name, nullptr, nullptr), "tensor_info");
                for (const auto& t : ts)
                    if (t.name == name) {
                        cad::check(cad_unet_set_tensor(h_, kind, i, t.value.data(), (int64_t)t.value.size()), name);
                        ++n;
                    }
            }
        }
        return n;
    }
    cad_unet* handle() const { return h_; }
    const cad::Workspace& workspace() const { return ws_; }

    float max_depth;

protected:
    BaselineUNetImpl(int model, int in_channels, int init_features, float max_depth_value, cad::Workspace ws)
        : max_depth(max_depth_value), ws_(ws) {
        cad_unet_desc d{in_channels, init_features, max_depth_value, ws.batch, ws.height, ws.width};
        cad::check(cad_unet_create_model(&d, model, ws.device, &h_), "cad_unet_create_model");
    }

private:
    std::vector<NamedTensor> fetch(int kind) const {
        const int cnt = kind == 0 ? cad_unet_num_params(h_) : cad_unet_num_buffers(h_);
        std::vector<NamedTensor> out;
        for (int i = 0; i < cnt; ++i) {
            const char* name;
            int nd;
            int64_t shp[4];
            cad::check(cad_unet_tensor_info(h_, kind, i, &name, &nd, shp), "tensor_info");
            NamedTensor t;
            t.name = name;
            t.shape.assign(shp, shp + nd);
            int64_t n = 1;
            for (int k = 0; k < nd; ++k) n *= shp[k];
            t.value.resize((size_t)n);
            cad::check(cad_unet_get_tensor(h_, kind, i, t.value.data(), n), "get_tensor");
            out.push_back(std::move(t));
        }
        return out;
    }
    cad::Workspace ws_;
    cad_unet* h_ = nullptr;
};

// IntrinsicsConditionedUNetImpl(in, f, camera_dim = 4, max_depth)   (intrinsics_unet.h:137-270):
// FiLMLayer(4, C) after every DoubleConv's first BN-ReLU; forward(x, camera_intrinsics (B,4)).
class IntrinsicsConditionedUNetImpl : public BaselineUNetImpl {
public:
    explicit IntrinsicsConditionedUNetImpl(int in_channels = 3, int init_features = 64, int camera_dim = 4,
                                           float max_depth_value = 10.0f, cad::Workspace ws = {},
                                           int model = CAD_MODEL_INTRINSICS_FILM)
        : BaselineUNetImpl(model, in_channels, init_features, max_depth_value, ws) {
        if (camera_dim != 4) throw std::runtime_error("camera_dim must be 4 ([fx, fy, cx, cy])");
    }
    // intrinsics: (B,4) [fx, fy, cx, cy] in pixels of the input (normalised on device, :252-268)
    DeviceTensor forward(const DeviceTensor& x, const DeviceTensor& intrinsics, void* stream = nullptr) {
        if (x.dim() != 4 || x.size(1) != 3) throw std::runtime_error("forward: expected (B,3,H,W)");
        if (intrinsics.dim() != 2 || intrinsics.size(0) != x.size(0) || intrinsics.size(1) != 4)
            throw std::runtime_error("forward: expected intrinsics (B,4)");
        DeviceTensor out = DeviceTensor::empty({x.size(0), 1, x.size(2), x.size(3)}, workspace().device);
        cad::check(cad_unet_forward_cam(handle(), x.data, intrinsics.data, out.data, (int)x.size(0), stream),
                   "forward");
        return out;
    }
    DeviceTensor operator()(const DeviceTensor& x, const DeviceTensor& intrinsics) { return forward(x, intrinsics); }
};

// Config-3 composite: enc1 = RayEnhancedConv(3, f, 4, use_rays) fed cat(x, rays(K)) (geometry_aware_network.h:17-65),
// FiLM blocks after; same forward(x, intrinsics) (rays derived on device from the intrinsics).
class RayConditionedUNetImpl : public IntrinsicsConditionedUNetImpl {
public:
    explicit RayConditionedUNetImpl(int in_channels = 3, int init_features = 64, int camera_dim = 4,
                                    float max_depth_value = 10.0f, cad::Workspace ws = {})
        : IntrinsicsConditionedUNetImpl(in_channels, init_features, camera_dim, max_depth_value, ws,
                                        CAD_MODEL_RAY_FILM) {}
};

// GeometryAwareNetworkImpl(in, f, camera_dim, max_depth, use_pcl, use_attention)
// (geometry_aware_network.h:201-347) and LightweightGeometryNetworkImpl(in, f, camera_dim, max_depth)
// (:355-440): forward(rgb, ray_directions (B,3,H,W), camera_intrinsics (B,4) [fx, fy, cx, cy]).
// Training: backward(dL/ddepth), then clip_grad_norm_ / adam_step on the model-owned slabs.
class GeometryAwareNetworkImpl {
public:
    explicit GeometryAwareNetworkImpl(int in_channels = 3, int init_features = 64, int camera_dim = 4,
                                      float max_depth_value = 10.0f, bool use_pcl = true, bool use_attention = true,
                                      cad::Workspace ws = {})
        : GeometryAwareNetworkImpl(CAD_GEONET_FULL, in_channels, init_features, camera_dim, max_depth_value, use_pcl,
                                   use_attention, ws) {}
    ~GeometryAwareNetworkImpl() { cad_geonet_destroy(h_); }
    GeometryAwareNetworkImpl(const GeometryAwareNetworkImpl&) = delete;
    GeometryAwareNetworkImpl& operator=(const GeometryAwareNetworkImpl&) = delete;

    DeviceTensor forward(const DeviceTensor& rgb, const DeviceTensor& ray_directions,
                         const DeviceTensor& camera_intrinsics, void* stream = nullptr) {
        if (rgb.dim() != 4 || rgb.size(1) != 3) throw std::runtime_error("forward: expected rgb (B,3,H,W)");
        if (ray_directions.dim() != 4 || ray_directions.size(0) != rgb.size(0) || ray_directions.size(1) != 3)
            throw std::runtime_error("forward: expected ray_directions (B,3,H,W)");
        if (camera_intrinsics.dim() != 2 || camera_intrinsics.size(0) != rgb.size(0) || camera_intrinsics.size(1) != 4)
            throw std::runtime_error("forward: expected camera_intrinsics (B,4)");
        DeviceTensor out = DeviceTensor::empty({rgb.size(0), 1, rgb.size(2), rgb.size(3)}, ws_.device);
        cad::check(cad_geonet_forward(h_, rgb.data, ray_directions.data, camera_intrinsics.data, out.data,
                                      (int)rgb.size(0), stream),
                   "forward");
        return out;
    }
    DeviceTensor operator()(const DeviceTensor& rgb, const DeviceTensor& rays, const DeviceTensor& intrinsics) {
        return forward(rgb, rays, intrinsics);
    }
    void backward(const DeviceTensor& ddepth, void* stream = nullptr) {
        cad::check(cad_geonet_backward(h_, ddepth.data, stream), "backward");
    }
    // torch::nn::utils::clip_grad_norm_(parameters(), max_norm) (prescale: 1/world after a gradient
    // all-reduce) and torch::optim::Adam(AdamOptions(lr).weight_decay(wd)).step()
    void clip_grad_norm_(float max_norm, float prescale = 1.0f, void* stream = nullptr) {
        cad::check(cad_geonet_clip_grad_norm(h_, max_norm, prescale, stream), "clip_grad_norm_");
    }
    void adam_step(float lr, float weight_decay, float beta1 = 0.9f, float beta2 = 0.999f, float eps = 1e-8f,
                   void* stream = nullptr) {
        cad::check(cad_geonet_adam_step(h_, lr, beta1, beta2, eps, weight_decay, stream), "adam_step");
    }
    int64_t count_parameters() const { return cad_geonet_count_parameters(h_); }
    void train(bool on = true) { cad::check(cad_geonet_train(h_, on ? 1 : 0), "train"); }
    void eval() { train(false); }
    std::vector<NamedTensor> named_parameters() const { return fetch(0); }
    std::vector<NamedTensor> named_buffers() const { return fetch(1); }
    int load(const std::vector<NamedTensor>& ts) {
        int n = 0;
        for (int kind = 0; kind < 2; ++kind)
            for (int i = 0; i < cad_geonet_num_tensors(h_, kind); ++i) {
                const char* name;
                cad::check(cad_geonet_tensor_info(h_, kind, i, &name, nullptr, nullptr), "tensor_info");
                for (const auto& t : ts)
                    if (t.name == name) {
                        cad::check(cad_geonet_set_tensor(h_, kind, i, t.value.data(), (int64_t)t.value.size()), name);
                        ++n;
                    }
            }
        return n;
    }
    cad_geonet* handle() const { return h_; }

    float max_depth;

protected:
    GeometryAwareNetworkImpl(int variant, int in_channels, int init_features, int camera_dim, float max_depth_value,
                             bool use_pcl, bool use_attention, cad::Workspace ws)
        : max_depth(max_depth_value), ws_(ws) {
        cad_geonet_desc d{variant, in_channels, init_features, camera_dim, max_depth_value, use_pcl ? 1 : 0,
                          use_attention ? 1 : 0, ws.batch, ws.height, ws.width};
        cad::check(cad_geonet_create(&d, ws.device, &h_), "cad_geonet_create");
    }

private:
    std::vector<NamedTensor> fetch(int kind) const {
        std::vector<NamedTensor> out;
        for (int i = 0; i < cad_geonet_num_tensors(h_, kind); ++i) {
            const char* name;
            int nd;
            int64_t shp[4];
            cad::check(cad_geonet_tensor_info(h_, kind, i, &name, &nd, shp), "tensor_info");
            NamedTensor t;
            t.name = name;
            t.shape.assign(shp, shp + nd);
            int64_t n = 1;
            for (int k = 0; k < nd; ++k) n *= shp[k];
            t.value.resize((size_t)n);
            cad::check(cad_geonet_get_tensor(h_, kind, i, t.value.data(), n), "get_tensor");
            out.push_back(std::move(t));
        }
        return out;
    }
    cad::Workspace ws_;
    cad_geonet* h_ = nullptr;
};

class LightweightGeometryNetworkImpl : public GeometryAwareNetworkImpl {
public:
    explicit LightweightGeometryNetworkImpl(int in_channels = 3, int init_features = 32, int camera_dim = 4,
                                            float max_depth_value = 10.0f, cad::Workspace ws = {})
        : GeometryAwareNetworkImpl(CAD_GEONET_LIGHT, in_channels, init_features, camera_dim, max_depth_value, true,
                                   true, ws) {}
};

class CombinedDepthLoss {
public:
    explicit CombinedDepthLoss(float si_weight = 1.0f, float grad_weight = 0.1f, float smooth_weight = 0.001f,
                               float reproj_weight = 0.01f, cad::Workspace ws = {})
        : w_{si_weight, grad_weight, smooth_weight, reproj_weight}, ws_(ws) {}
    ~CombinedDepthLoss() {
        cad_loss_destroy(with_);
        cad_loss_destroy(without_);
    }
    CombinedDepthLoss(const CombinedDepthLoss&) = delete;
    CombinedDepthLoss& operator=(const CombinedDepthLoss&) = delete;

    // forwardWithIntrinsics(pred, gt, image, intrinsics, valid_mask) (depth_loss.h:416-433): returns the
    // 5-float device tensor {total, si, grad, smooth, reproj}; dL/dpred is left in dpred().  valid_mask
    // replaces gt > 1e-6 in the SI and reprojection terms (grad matching ignores it, :137).
    DeviceTensor forwardWithIntrinsics(const DeviceTensor& pred, const DeviceTensor& gt, const DeviceTensor& image,
                                       const DeviceTensor& intrinsics,
                                       const std::optional<cad::DeviceMask>& valid_mask = std::nullopt,
                                       void* stream = nullptr) {
        return run(get(true), pred, gt, image, intrinsics, valid_mask, stream);
    }
    // forward(pred, gt, image, valid_mask) (depth_loss.h:390-404): SI + grad + smooth, no reprojection
    DeviceTensor forward(const DeviceTensor& pred, const DeviceTensor& gt, const DeviceTensor& image,
                         const std::optional<cad::DeviceMask>& valid_mask = std::nullopt, void* stream = nullptr) {
        return run(get(false), pred, gt, image, identity_K(pred.size(0)), valid_mask, stream);
    }
    std::map<std::string, float> getComponentsWithIntrinsics(const DeviceTensor& pred, const DeviceTensor& gt,
                                                             const DeviceTensor& image, const DeviceTensor& K,
                                                             const std::optional<cad::DeviceMask>& valid_mask = std::nullopt) {
        DeviceTensor l = forwardWithIntrinsics(pred, gt, image, K, valid_mask);
        auto v = l.to_host();
        return {{"si_loss", v[1]}, {"grad_loss", v[2]}, {"smooth_loss", v[3]}, {"reproj_loss", v[4]}};
    }
    std::map<std::string, float> getComponents(const DeviceTensor& pred, const DeviceTensor& gt,
                                               const DeviceTensor& image,
                                               const std::optional<cad::DeviceMask>& valid_mask = std::nullopt) {
        DeviceTensor l = forward(pred, gt, image, valid_mask);
        auto v = l.to_host();
        return {{"si_loss", v[1]}, {"grad_loss", v[2]}, {"smooth_loss", v[3]}};
    }
    const DeviceTensor& dpred() const { return dpred_; }

private:
    cad_loss* get(bool with_reproj) {
        cad_loss*& h = with_reproj ? with_ : without_;
        if (!h)
            cad::check(cad_loss_create(w_[0], w_[1], w_[2], with_reproj ? w_[3] : 0.f, ws_.batch, ws_.height,
                                       ws_.width, ws_.device, &h), "CombinedDepthLoss");
        return h;
    }
    DeviceTensor run(cad_loss* h, const DeviceTensor& pred, const DeviceTensor& gt, const DeviceTensor& image,
                     const DeviceTensor& K, const std::optional<cad::DeviceMask>& mask, void* stream) {
        if (mask && mask->numel() != pred.numel()) throw std::runtime_error("valid_mask must be (B,1,H,W)");
        if (dpred_.numel() != pred.numel()) dpred_ = DeviceTensor::empty(pred.shape, ws_.device);
        DeviceTensor l = DeviceTensor::empty({5}, ws_.device);
        cad::check(cad_loss_forward_backward_masked(h, pred.data, gt.data, image.data, K.data, mask ? mask->data : nullptr,
                                                    (int)pred.size(0), l.data, dpred_.data, stream),
                   "forwardWithIntrinsics");
        return l;
    }
    // the kernels take intrinsics for their pixel grid even when the reprojection weight is 0
    const DeviceTensor& identity_K(int64_t B) {
        if (eye_.numel() < B * 9) {
            std::vector<float> h((size_t)(B * 9), 0.f);
            for (int64_t b = 0; b < B; ++b) h[b * 9] = h[b * 9 + 4] = h[b * 9 + 8] = 1.f;
            eye_ = DeviceTensor::from_host(h.data(), {B, 3, 3}, ws_.device);
        }
        return eye_;
    }
    float w_[4];
    cad::Workspace ws_;
    cad_loss* with_ = nullptr;
    cad_loss* without_ = nullptr;
    DeviceTensor dpred_, eye_;
};

namespace optim {
class Adam {   // torch::optim::Adam(params, AdamOptions(lr).weight_decay(wd)) — coupled L2
public:
    Adam(BaselineUNetImpl& model, float lr = 1e-3f, float weight_decay = 0.f, float beta1 = 0.9f,
         float beta2 = 0.999f, float eps = 1e-8f) {
        cad_adam_opts o{lr, beta1, beta2, eps, weight_decay};
        cad::check(cad_adam_create(model.handle(), &o, &h_), "Adam");
    }
    ~Adam() { cad_adam_destroy(h_); }
    Adam(const Adam&) = delete;
    Adam& operator=(const Adam&) = delete;
    void zero_grad() {}   // every backward overwrites the gradient slab
    void step(void* stream = nullptr) { cad::check(cad_adam_step(h_, stream), "Adam::step"); }
    void set_lr(float lr) { cad::check(cad_adam_set_lr(h_, lr), "set_lr"); }
    int64_t step_count() const { return cad_adam_step_count(h_); }
    cad_adam* handle() const { return h_; }

private:
    cad_adam* h_ = nullptr;
};
}  // namespace optim

// torch::nn::utils::clip_grad_norm_(model->parameters(), max_norm) -> total norm (synchronises).
// prescale scales the gradients first (1/world after a SUM all-reduce: the norm of the mean gradient)
inline double clip_grad_norm_(BaselineUNetImpl& model, double max_norm, void* stream = nullptr, double prescale = 1.0) {
    cad::check(cad_clip_grad_norm(model.handle(), (float)max_norm, (float)prescale, stream), "clip_grad_norm_");
    float n = 0.f;
    cad::check(cad_unet_last_grad_norm(model.handle(), &n, stream), "clip_grad_norm_");
    return n;
}

// torch::save(model_, path) / torch::load(model, path) (tensorboard_trainer_enhanced.h:656-662): the
// TorchScript archive LibTorch writes for the module; either side reads the other's files.
inline void save(const BaselineUNetImpl& model, const std::string& path) {
    cad::check(cad_unet_save_torch(model.handle(), path.c_str()), "torch::save");
}
inline void load(BaselineUNetImpl& model, const std::string& path) {
    cad::check(cad_unet_load_torch(model.handle(), path.c_str()), "torch::load");
}

// Data-parallel replicas over RCCL (new: the reference is single-device).  One
// process per GPU; rank 0 draws the id (unique_id()) and every rank builds the communicator from it.
namespace distributed {
using UniqueId = std::array<uint8_t, CAD_COMM_ID_BYTES>;
class Communicator {
public:
    static UniqueId unique_id() {
        UniqueId id{};
        cad::check(cad_comm_get_unique_id(id.data()), "cad_comm_get_unique_id");
        return id;
    }
    Communicator(const UniqueId& id, int world_size, int rank, int device) {
        cad::check(cad_comm_create(id.data(), world_size, rank, device, &h_), "cad_comm_create");
    }
    ~Communicator() { cad_comm_destroy(h_); }
    Communicator(const Communicator&) = delete;
    Communicator& operator=(const Communicator&) = delete;
    int rank() const { return cad_comm_rank(h_); }
    int size() const { return cad_comm_size(h_); }
    void allreduce(float* buf, int64_t count, int op = CAD_REDUCE_SUM, void* stream = nullptr) {
        cad::check(cad_comm_allreduce(h_, buf, count, op, stream), "cad_comm_allreduce");
    }
    // identical replicas: rank `root`'s parameters everywhere
    void broadcast_parameters(BaselineUNetImpl& m, int root = 0, void* stream = nullptr) {
        cad::check(cad_comm_broadcast_params(m.handle(), h_, root, stream), "cad_comm_broadcast_params");
    }
    // loss.backward() with the bucketed gradient all-reduce overlapped (decoder-first buckets)
    void backward_allreduce(BaselineUNetImpl& m, const DeviceTensor& ddepth, int64_t bucket_elems = 25 << 18,
                            void* stream = nullptr) {
        cad::check(cad_unet_backward_allreduce(m.handle(), h_, ddepth.data, bucket_elems, stream),
                   "cad_unet_backward_allreduce");
    }
    cad_comm* handle() const { return h_; }

private:
    cad_comm* h_ = nullptr;
};
}  // namespace distributed

// computeDepthMetrics (tensorboard_trainer_enhanced.h:400-439), averaged over the batch
struct DepthMetrics {
    float abs_rel = 0, sq_rel = 0, rmse = 0, rmse_log = 0, a1 = 0, a2 = 0, a3 = 0;
};
inline DepthMetrics computeDepthMetrics(const DeviceTensor& pred, const DeviceTensor& gt, void* stream = nullptr) {
    float o[7];
    cad::check(cad_depth_metrics(pred.data, gt.data, (int)pred.size(0), (int)pred.size(2), (int)pred.size(3), o, stream),
               "computeDepthMetrics");
    return {o[0], o[1], o[2], o[3], o[4], o[5], o[6]};
}

}  // namespace camera_aware_depth

#endif  // CAD_CAD_HPP

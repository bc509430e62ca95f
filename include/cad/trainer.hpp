// trainer.hpp — header-only C++ drop-in for the reference's training driver, over cad.hpp / cad.h.
//
//   camera_aware_depth::AugmentationConfig          src/data/sunrgbd_loader.h:31-46
//   camera_aware_depth::SunRGBDLoader               src/data/sunrgbd_loader.h:60-128, sunrgbd_loader.cpp:13-78
//   camera_aware_depth::TensorBoardTrainerEnhanced  src/training/tensorboard_trainer_enhanced.h:35-700
//
// Same class names, Config / ValidationMetrics fields, constructor and train(train, val) as the
// reference; the step is the reference's (zero_grad, forward, forwardWithIntrinsics, backward,
// clip_grad_norm_, Adam.step, enhanced.h:287-304) on the MI355X through libcad.  Batches come from the
// loader's prefetch ring (cad_loader: decode threads, pinned double-buffered upload, device resize and
// augmentation) instead of getBatch + torch::stack.  Deliberate differences:
//   * TensorBoard event files are a CSV of scalars (<log_dir>/tensorboard_scalars.csv); images and
//     histograms are not written (gradients/norm|max|min scalars are);
//   * with a distributed::Communicator the step is data-parallel (the reference is single-device):
//     rank r trains its batch_size-slice of every global batch, gradients are SUM-all-reduced in
//     buckets overlapped with the backward and clipped as the mean; rank 0 validates, logs and saves;
//   * logLossComponents reads sample 0 without augmentation (the reference's getSample(0) draws from
//     the augmentation rng).
#ifndef CAD_TRAINER_HPP
#define CAD_TRAINER_HPP

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <ctime>
#include <filesystem>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <limits>
#include <sstream>
#include <thread>

#include "cad.hpp"

namespace camera_aware_depth {

struct AugmentationConfig {   // sunrgbd_loader.h:31-46 (saturation / hue are parsed, unused by augmentSample)
    bool enable_random_crop = true;
    float crop_scale_min = 0.7f;
    float crop_scale_max = 1.0f;
    bool enable_horizontal_flip = true;
    float horizontal_flip_prob = 0.5f;
    bool enable_color_jitter = true;
    float brightness_delta = 0.2f;
    float contrast_delta = 0.2f;
    float saturation_delta = 0.2f;
    float hue_delta = 0.1f;
    int random_seed = 42;
};

// SUN RGB-D samples from the JSON manifest (valid entries of the allowed sensor types with an
// intrinsics.txt, paths relative to the working directory — data_dir and split are kept but unused,
// as in the reference), resized to the target dimensions (default 480x640, :21-22).
class SunRGBDLoader {
public:
    SunRGBDLoader(const std::string& data_dir, const std::string& manifest_path, const std::string& split)
        : data_dir_(data_dir), manifest_(manifest_path), split_(split) {
        open();
    }
    // n procedurally generated samples of height x width (the synthetic dataset; no files)
    static std::shared_ptr<SunRGBDLoader> synthetic(int64_t n, int height, int width, uint32_t seed = 0) {
        std::shared_ptr<SunRGBDLoader> L(new SunRGBDLoader());
        cad_dataset* d = nullptr;
        cad::check(cad_dataset_synthetic(n, height, width, seed, &d), "synthetic dataset");
        L->ds_.reset(d, cad_dataset_destroy);
        L->h_ = height;
        L->w_ = width;
        return L;
    }
    size_t size() const { return (size_t)cad_dataset_size(ds_.get()); }
    void enableAugmentation(const AugmentationConfig& c) { aug_ = c; augment_ = true; rings_.clear(); }
    void disableAugmentation() { augment_ = false; rings_.clear(); }
    bool augmentation_enabled() const { return augment_; }
    void setTargetDimensions(int height, int width) { h_ = height; w_ = width; rings_.clear(); }
    int target_height() const { return h_; }
    int target_width() const { return w_; }
    void filterBySensorType(const std::vector<std::string>& sensor_types) {
        if (manifest_.empty()) throw std::runtime_error("filterBySensorType: the synthetic dataset has no sensors");
        sensors_ = sensor_types;
        open();
    }
    const std::string& manifest_path() const { return manifest_; }
    cad_dataset* handle() const { return ds_.get(); }

    // The batch pipeline behind getBatch: a prefetch ring of `batch`-sample batches on `device`
    // (augmented when augmentation is enabled and `augment`), created on first use.
    cad_loader* ring(int batch, int device, bool augment) {
        const bool aug = augment && augment_;
        const auto key = std::make_tuple(batch, device, aug);
        for (auto& r : rings_)
            if (r.first == key) return r.second.get();
        cad_aug_config ac{};
        ac.enable_random_crop = aug_.enable_random_crop;
        ac.crop_scale_min = aug_.crop_scale_min;
        ac.crop_scale_max = aug_.crop_scale_max;
        ac.enable_horizontal_flip = aug_.enable_horizontal_flip;
        ac.horizontal_flip_prob = aug_.horizontal_flip_prob;
        ac.enable_color_jitter = aug_.enable_color_jitter;
        ac.brightness_delta = aug_.brightness_delta;
        ac.contrast_delta = aug_.contrast_delta;
        const int threads = (int)std::max(2u, std::min(8u, std::thread::hardware_concurrency()));
        cad_loader* L = nullptr;
        cad::check(cad_loader_create(ds_.get(), batch, h_, w_, aug ? &ac : nullptr, (uint32_t)aug_.random_seed, threads,
                                     2, device, &L),
                   "SunRGBDLoader");
        rings_.emplace_back(key, std::shared_ptr<cad_loader>(L, cad_loader_destroy));
        return L;
    }

private:
    SunRGBDLoader() = default;
    void open() {
        std::vector<const char*> s;
        for (const auto& x : sensors_) s.push_back(x.c_str());
        cad_dataset* d = nullptr;
        cad::check(cad_dataset_open(manifest_.c_str(), s.empty() ? nullptr : s.data(), (int)s.size(), &d), "SunRGBDLoader");
        ds_.reset(d, cad_dataset_destroy);
        rings_.clear();
    }
    std::string data_dir_, manifest_, split_;
    std::vector<std::string> sensors_;
    std::shared_ptr<cad_dataset> ds_;
    int h_ = 480, w_ = 640;
    bool augment_ = false;
    AugmentationConfig aug_{};
    std::vector<std::pair<std::tuple<int, int, bool>, std::shared_ptr<cad_loader>>> rings_;
};

// .cadckpt: named parameters and buffers (reference layout) + the Adam state the reference never
// saves (moments, step count) — a full resume.  torch::save archives (.pt) carry the weights only.
inline void save_training_state(const std::string& path, BaselineUNetImpl& m, optim::Adam& opt) {
    std::ofstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot write checkpoint " + path);
    auto ps = m.named_parameters();
    auto bs = m.named_buffers();
    ps.insert(ps.end(), bs.begin(), bs.end());
    f.write("CADCKPT1", 8);
    const int32_t n = (int32_t)ps.size();
    f.write((const char*)&n, 4);
    for (auto& t : ps) {
        const int32_t ln = (int32_t)t.name.size(), nd = (int32_t)t.shape.size();
        f.write((const char*)&ln, 4);
        f.write(t.name.data(), ln);
        f.write((const char*)&nd, 4);
        f.write((const char*)t.shape.data(), 8 * nd);
        f.write((const char*)t.value.data(), 4 * (int64_t)t.value.size());
    }
    float *mp, *vp;
    int64_t nflat;
    cad::check(cad_unet_flat(m.handle(), nullptr, nullptr, &nflat), "flat");
    cad::check(cad_adam_state(opt.handle(), &mp, &vp), "adam_state");
    std::vector<float> buf((size_t)nflat);
    const int64_t step = opt.step_count();
    f.write("ADAM", 4);
    f.write((const char*)&step, 8);
    f.write((const char*)&nflat, 8);
    for (float* src : {mp, vp}) {
        cad::check(cad_memcpy(buf.data(), src, 4 * nflat, 1, nullptr), "d2h");
        f.write((const char*)buf.data(), 4 * nflat);
    }
}

inline void load_training_state(const std::string& path, BaselineUNetImpl& m, optim::Adam& opt) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("Cannot open checkpoint: " + path);
    char magic[8];
    f.read(magic, 8);
    if (!f || std::memcmp(magic, "CADCKPT1", 8) != 0) throw std::runtime_error("not a .cadckpt file: " + path);
    int32_t n;
    f.read((char*)&n, 4);
    std::vector<NamedTensor> ts((size_t)std::max(0, n));
    for (auto& t : ts) {
        int32_t ln, nd;
        f.read((char*)&ln, 4);
        t.name.resize((size_t)ln);
        f.read(&t.name[0], ln);
        f.read((char*)&nd, 4);
        t.shape.resize((size_t)nd);
        f.read((char*)t.shape.data(), 8 * nd);
        int64_t cnt = 1;
        for (auto s : t.shape) cnt *= s;
        t.value.resize((size_t)cnt);
        f.read((char*)t.value.data(), 4 * cnt);
    }
    if (!f || m.load(ts) != n) throw std::runtime_error("checkpoint does not match the model: " + path);
    char tag[4];
    if (f.read(tag, 4) && std::memcmp(tag, "ADAM", 4) == 0) {
        int64_t step, nflat, mine;
        f.read((char*)&step, 8);
        f.read((char*)&nflat, 8);
        float *mp, *vp;
        cad::check(cad_unet_flat(m.handle(), nullptr, nullptr, &mine), "flat");
        if (nflat != mine) throw std::runtime_error("optimizer state size mismatch in " + path);
        cad::check(cad_adam_state(opt.handle(), &mp, &vp), "adam_state");
        std::vector<float> buf((size_t)nflat);
        for (float* dst : {mp, vp}) {
            f.read((char*)buf.data(), 4 * nflat);
            cad::check(cad_memcpy(dst, buf.data(), 4 * nflat, 0, nullptr), "h2d");
        }
        cad::check(cad_adam_set_step_count(opt.handle(), step), "set_step");
    }
}

class TensorBoardTrainerEnhanced {
public:
    struct Config {   // enhanced.h:37-63
        int num_epochs = 50;
        int batch_size = 8;
        float learning_rate = 1e-4f;
        float weight_decay = 1e-5f;
        bool use_grad_clip = true;
        float grad_clip_value = 1.0f;
        int val_interval = 10;
        int log_interval = 10;
        int save_interval = 5;
        int viz_interval = 1;
        int num_viz_samples = 4;
        int histogram_interval = 5;
        int profiler_interval = 0;
        std::string checkpoint_dir = "./checkpoints";
        std::string log_dir = "./logs";
        std::string tensorboard_dir = "./runs";
        std::string experiment_name = "experiment";
        int device = 0;              // torch::Device: the MI355X ordinal
        bool tensorboard = true;     // write <log_dir>/tensorboard_scalars.csv
        bool save_optimizer = true;  // also write <name>_epoch_N.cadckpt next to each .pt
        int64_t bucket_elems = 25 << 18;   // data-parallel gradient buckets (25 MB)
    };

    struct ValidationMetrics {   // enhanced.h:65-74
        float loss = 0.0f, abs_rel = 0.0f, sq_rel = 0.0f, rmse = 0.0f, rmse_log = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
    };

    // model and model_impl are the same network (the reference passes the Module and its Impl)
    TensorBoardTrainerEnhanced(std::shared_ptr<BaselineUNetImpl> model, std::shared_ptr<BaselineUNetImpl> model_impl,
                               std::shared_ptr<CombinedDepthLoss> loss_fn, const Config& config,
                               std::shared_ptr<distributed::Communicator> comm = nullptr)
        : model_(model_impl ? model_impl : model), loss_fn_(std::move(loss_fn)), config_(config), comm_(std::move(comm)) {
        if (!model_ || !loss_fn_) throw std::runtime_error("TensorBoardTrainerEnhanced: model and loss are required");
        rank_ = comm_ ? comm_->rank() : 0;
        world_ = comm_ ? comm_->size() : 1;
        optimizer_ = std::make_shared<optim::Adam>(*model_, config_.learning_rate, config_.weight_decay);
        if (lead()) {
            std::filesystem::create_directories(config_.checkpoint_dir);
            std::filesystem::create_directories(config_.log_dir);
            train_log_.open(config_.log_dir + "/training.log", std::ios::app);
            metrics_csv_.open(config_.log_dir + "/metrics.csv", std::ios::app);
            if (metrics_csv_.tellp() == 0)   // :111-115
                metrics_csv_ << "epoch,step,train_loss,val_loss,abs_rel,sq_rel,rmse,rmse_log,a1,a2,a3,learning_rate,time_elapsed\n";
            if (config_.tensorboard) {
                tb_.open(config_.log_dir + "/tensorboard_scalars.csv", std::ios::app);
                if (tb_.tellp() == 0) tb_ << "tag,step,value\n";
            }
        }
        if (comm_) comm_->broadcast_parameters(*model_, 0);   // identical replicas
    }

    optim::Adam& optimizer() { return *optimizer_; }
    int64_t global_step() const { return global_step_; }
    // resume: parameters, BN buffers and the Adam state (.cadckpt), or the weights of a torch::save
    // archive (.pt: ours or the reference's; the optimizer starts fresh)
    void loadCheckpoint(const std::string& path) {
        if (path.size() >= 3 && path.compare(path.size() - 3, 3, ".pt") == 0) load(*model_, path);
        else load_training_state(path, *model_, *optimizer_);
        if (comm_) comm_->broadcast_parameters(*model_, 0);
    }
    void saveTrainingState(const std::string& path) { save_training_state(path, *model_, *optimizer_); }

    // enhanced.h:142-240.  Epochs continue after a resumed optimizer step count (whole epochs done).
    void train(std::shared_ptr<SunRGBDLoader> train_loader, std::shared_ptr<SunRGBDLoader> val_loader = nullptr) {
        if (!train_loader) throw std::runtime_error("train: no training loader");
        const int nb = steps_per_epoch(train_loader->size());
        if (nb < 1) throw std::runtime_error("fewer training samples than one global batch");
        logMessage("=== Starting Training (MI355X) ===");
        logMessage("Train samples: " + std::to_string(train_loader->size()));
        if (val_loader) logMessage("Val samples: " + std::to_string(val_loader->size()));
        logMessage("Batch size: " + std::to_string(config_.batch_size) +
                   (world_ > 1 ? " per rank x " + std::to_string(world_) + " ranks" : std::string()));
        logMessage("Epochs: " + std::to_string(config_.num_epochs));
        if (tb_) {   // logHyperparameters / logModelArchitecture (:576-615)
            tb_ << "hparams/learning_rate,0," << config_.learning_rate << "\nhparams/batch_size,0," << config_.batch_size
                << "\nhparams/weight_decay,0," << config_.weight_decay << "\nhparams/grad_clip_value,0,"
                << config_.grad_clip_value << "\nhparams/num_epochs,0," << config_.num_epochs
                << "\nmodel/total_parameters,0," << model_->count_parameters() << "\n";
        }
        const auto t0 = std::chrono::steady_clock::now();
        global_step_ = optimizer_->step_count() / nb * nb;
        for (int epoch = 1 + (int)(optimizer_->step_count() / nb); epoch <= config_.num_epochs; ++epoch) {
            const auto te = std::chrono::steady_clock::now();
            if (lead()) std::cout << "\n" << std::string(60, '=') << "\nEpoch " << epoch << "/" << config_.num_epochs << "\n";
            const float train_loss = trainEpoch(*train_loader, nb, (int)global_step_, epoch);
            if (lead()) {
                scalar("loss/train", train_loss, epoch);
                scalar("training/learning_rate", config_.learning_rate, epoch);
                logLossComponents(*train_loader, epoch);
                scalar("training/epoch_time_seconds",
                       (double)std::chrono::duration_cast<std::chrono::seconds>(std::chrono::steady_clock::now() - te).count(),
                       epoch);
            }
            ValidationMetrics vm;
            if (lead() && val_loader && config_.val_interval > 0 && epoch % config_.val_interval == 0) {
                vm = validateEpoch(*val_loader, epoch);
                scalar("loss/val", vm.loss, epoch);
                scalar("metrics/abs_rel", vm.abs_rel, epoch);
                scalar("metrics/sq_rel", vm.sq_rel, epoch);
                scalar("metrics/rmse", vm.rmse, epoch);
                scalar("metrics/rmse_log", vm.rmse_log, epoch);
                scalar("metrics/a1", vm.a1, epoch);
                scalar("metrics/a2", vm.a2, epoch);
                scalar("metrics/a3", vm.a3, epoch);
            }
            if (lead() && config_.histogram_interval > 0 && epoch % config_.histogram_interval == 0)
                logGradientStatistics(epoch);
            if (lead() && config_.save_interval > 0 && epoch % config_.save_interval == 0) saveCheckpoint(epoch);
            const long total = (long)std::chrono::duration_cast<std::chrono::seconds>(std::chrono::steady_clock::now() - t0).count();
            if (lead()) {
                logEpochMetrics(epoch, (int)global_step_, train_loss, vm, total);
                scalar("training/total_time_seconds", (double)total, epoch);
            }
            global_step_ += nb;   // :233
        }
        if (lead()) {
            save(*model_, config_.checkpoint_dir + "/final_model.pt");   // production_trainer.h:323-330
            if (config_.save_optimizer) saveTrainingState(config_.checkpoint_dir + "/final_model.cadckpt");
            logMessage("=== Training Complete ===");
        }
    }

    // per-rank batches of an epoch: global batch bi = samples [bi*B*world, (bi+1)*B*world); with more
    // than one rank the last partial global batch is dropped (every replica steps together)
    int steps_per_epoch(size_t n) const {
        const int64_t B = config_.batch_size;
        return world_ > 1 ? (int)((int64_t)n / (B * world_)) : (int)(((int64_t)n + B - 1) / B);
    }

private:
    bool lead() const { return rank_ == 0; }
    bool conditioned() const { return cad_unet_model(model_->handle()) != CAD_MODEL_BASELINE; }

    void ensure_buffers(const SunRGBDLoader& L) {
        const int B = config_.batch_size, H = L.target_height(), W = L.target_width();
        if (rgb_.numel() == (int64_t)B * 3 * H * W) return;
        const int d = config_.device;
        rgb_ = DeviceTensor::empty({B, 3, H, W}, d);
        gt_ = DeviceTensor::empty({B, 1, H, W}, d);
        K_ = DeviceTensor::empty({B, 3, 3}, d);
        pred_ = DeviceTensor::empty({B, 1, H, W}, d);
        cam_ = DeviceTensor::empty({B, 4}, d);
    }
    int next(cad_loader* ring, int expect) {
        const int n = cad_loader_next(ring, rgb_.data, gt_.data, K_.data, nullptr);
        if (n < 0) throw std::runtime_error(std::string("data loader: ") + cad_last_error());
        if (expect >= 0 && n != expect)
            throw std::runtime_error("data loader: batch of " + std::to_string(n) + ", expected " + std::to_string(expect));
        for (DeviceTensor* t : {&rgb_, &gt_, &K_, &pred_, &cam_}) t->shape[0] = n;
        return n;
    }
    // model_impl_->forward(rgb) (baseline) / forward(rgb, intrinsics) (the FiLM models, camera from K)
    void forward() {
        const int n = (int)rgb_.size(0);
        if (conditioned()) {
            cad::check(cad_camera_from_K(K_.data, n, cam_.data, nullptr), "camera_from_K");
            cad::check(cad_unet_forward_cam(model_->handle(), rgb_.data, cam_.data, pred_.data, n, nullptr), "forward");
        } else {
            model_->forward_into(rgb_, pred_);
        }
    }

    float trainEpoch(SunRGBDLoader& L, int nb, int global_step, int epoch) {   // :257-334
        (void)epoch;
        ensure_buffers(L);
        model_->train();
        const int B = config_.batch_size;
        const int64_t n = (int64_t)L.size();
        std::vector<int64_t> order;   // this rank's samples, in step order
        for (int bi = 0; bi < nb; ++bi) {
            const int64_t first = (int64_t)bi * B * world_ + (int64_t)rank_ * B;
            for (int64_t j = first; j < std::min<int64_t>(first + B, n); ++j) order.push_back(j);
        }
        cad_loader* ring = L.ring(B, config_.device, true);
        cad::check(cad_loader_start_epoch(ring, order.data(), (int64_t)order.size()), "start epoch");
        double total = 0.0;
        int64_t seen = 0;
        for (int bi = 0; bi < nb; ++bi) {
            const int64_t first = (int64_t)bi * B * world_ + (int64_t)rank_ * B;
            const int bs = (int)std::min<int64_t>(B, n - first);
            next(ring, bs);
            optimizer_->zero_grad();
            forward();
            DeviceTensor l = loss_fn_->forwardWithIntrinsics(pred_, gt_, rgb_, K_);
            if (comm_) comm_->backward_allreduce(*model_, loss_fn_->dpred(), config_.bucket_elems);
            else model_->backward(loss_fn_->dpred());
            // clip_grad_norm_ on the mean gradient (the SUM all-reduce's 1/world folded in)
            double gnorm = 0.0;
            if (config_.use_grad_clip) gnorm = clip_grad_norm_(*model_, config_.grad_clip_value, nullptr, 1.0 / world_);
            else cad::check(cad_clip_grad_norm(model_->handle(), INFINITY, 1.f / world_, nullptr), "prescale");
            optimizer_->step();
            if (comm_) comm_->allreduce(l.data, 5);   // the logged loss: mean over replicas
            const float lv = l.to_host()[0] / world_;   // loss.item<float>() (:307)
            if (!std::isfinite(lv)) throw std::runtime_error("non-finite loss at step " + std::to_string(global_step + bi));
            total += (double)lv * bs * world_;
            seen += (int64_t)bs * world_;
            if (lead() && (bi + 1) % std::max(1, config_.log_interval) == 0) {   // :313-319
                scalar("batch_loss/train", lv, global_step + bi);
                if (!config_.use_grad_clip) gnorm = clip_grad_norm_(*model_, INFINITY);   // computeGradientNorm
                scalar("training/gradient_norm", gnorm, global_step + bi);
            }
            if (lead() && ((bi + 1) % std::max(1, config_.log_interval) == 0 || bi == nb - 1))
                std::cout << "\r  [" << std::setw(3) << (100 * (bi + 1) / nb) << "%] Batch " << (bi + 1) << "/" << nb
                          << " | Loss: " << std::fixed << std::setprecision(4) << lv << std::flush;
        }
        if (lead()) std::cout << std::endl;
        return (float)(total / std::max<int64_t>(1, seen));
    }

    // validateEpoch (:339-395): the first min(500, size) samples one at a time in eval mode; loss and
    // computeDepthMetrics averaged per sample
    ValidationMetrics validateEpoch(SunRGBDLoader& L, int epoch) {
        (void)epoch;
        ensure_buffers(L);
        model_->eval();
        ValidationMetrics m;
        const int64_t ns = std::min<int64_t>(500, (int64_t)L.size());
        cad_loader* ring = L.ring(1, config_.device, false);
        cad::check(cad_loader_start_epoch(ring, nullptr, ns), "validation");
        int count = 0;
        for (int64_t i = 0; i < ns; ++i) {
            next(ring, 1);
            forward();
            DeviceTensor l = loss_fn_->forwardWithIntrinsics(pred_, gt_, rgb_, K_);
            const DepthMetrics s = computeDepthMetrics(pred_, gt_);
            m.loss += l.to_host()[0];
            m.abs_rel += s.abs_rel; m.sq_rel += s.sq_rel; m.rmse += s.rmse; m.rmse_log += s.rmse_log;
            m.a1 += s.a1; m.a2 += s.a2; m.a3 += s.a3;
            ++count;
        }
        if (count)
            for (float* p : {&m.loss, &m.abs_rel, &m.sq_rel, &m.rmse, &m.rmse_log, &m.a1, &m.a2, &m.a3}) *p /= count;
        model_->train();
        return m;
    }

    void logLossComponents(SunRGBDLoader& L, int epoch) {   // :475-501
        if (!tb_ || L.size() == 0) return;
        ensure_buffers(L);
        model_->eval();
        cad_loader* ring = L.ring(1, config_.device, false);
        cad::check(cad_loader_start_epoch(ring, nullptr, 1), "loss components");
        next(ring, 1);
        forward();
        auto c = loss_fn_->getComponentsWithIntrinsics(pred_, gt_, rgb_, K_);
        for (const char* k : {"si_loss", "grad_loss", "smooth_loss", "reproj_loss"})
            scalar(std::string("loss_components/") + k, c[k], epoch);
        model_->train();
    }

    void logGradientStatistics(int epoch) {   // :523-555 (scalars; no histograms)
        if (!tb_) return;
        double norm = 0.0;
        float mx = 0.f, mn = std::numeric_limits<float>::max();
        for (const auto& g : model_->named_grads()) {
            double s = 0.0;
            for (float v : g.value) { s += (double)v * v; mx = std::max(mx, v); mn = std::min(mn, v); }
            norm += s;
        }
        scalar("gradients/norm", std::sqrt(norm), epoch);
        scalar("gradients/max", mx, epoch);
        scalar("gradients/min", mn, epoch);
    }

    void logEpochMetrics(int epoch, int step, float train_loss, const ValidationMetrics& v, long elapsed) {   // :620-651
        std::stringstream ss;
        ss << "Epoch " << epoch << " | Train Loss: " << std::fixed << std::setprecision(4) << train_loss;
        if (v.loss > 0)
            ss << " | Val Loss: " << v.loss << " | abs_rel: " << v.abs_rel << " | rmse: " << v.rmse
               << " | a1: " << std::setprecision(3) << v.a1;
        ss << " | Time: " << elapsed << "s";
        logMessage(ss.str());
        metrics_csv_ << epoch << "," << step << "," << train_loss << "," << v.loss << "," << v.abs_rel << "," << v.sq_rel
                     << "," << v.rmse << "," << v.rmse_log << "," << v.a1 << "," << v.a2 << "," << v.a3 << ","
                     << config_.learning_rate << "," << elapsed << "\n";
        metrics_csv_.flush();
    }

    void saveCheckpoint(int epoch) {   // :656-662: torch::save(model_, <dir>/<experiment>_epoch_N.pt)
        const std::string stem = config_.checkpoint_dir + "/" + config_.experiment_name + "_epoch_" + std::to_string(epoch);
        save(*model_, stem + ".pt");
        if (config_.save_optimizer) saveTrainingState(stem + ".cadckpt");
        logMessage("Checkpoint saved: " + stem + ".pt");
    }

    void scalar(const std::string& tag, double v, int64_t step) {
        if (tb_) tb_ << tag << "," << step << "," << v << "\n";
    }
    void logMessage(const std::string& msg) {   // :667-682
        if (!lead()) return;
        const std::time_t t = std::time(nullptr);
        std::stringstream ts;
        ts << "[" << std::put_time(std::localtime(&t), "%Y-%m-%d %H:%M:%S") << "] " << msg;
        std::cout << ts.str() << std::endl;
        if (train_log_.is_open()) {
            train_log_ << ts.str() << "\n";
            train_log_.flush();
        }
    }

    std::shared_ptr<BaselineUNetImpl> model_;
    std::shared_ptr<CombinedDepthLoss> loss_fn_;
    std::shared_ptr<optim::Adam> optimizer_;
    Config config_;
    std::shared_ptr<distributed::Communicator> comm_;
    int rank_ = 0, world_ = 1;
    int64_t global_step_ = 0;
    std::ofstream train_log_, metrics_csv_, tb_;
    DeviceTensor rgb_, gt_, K_, pred_, cam_;
};

// The same training loop (enhanced.h:142-240, 257-395) for the geometry-aware networks
// (geometry_aware_network.h: GeometryAwareNetworkImpl / LightweightGeometryNetworkImpl), fed the
// loader's batch as the reference's forward takes it: rgb, RayDirectionComputer's rays (a18) and the
// (B,4) intrinsics (a15).  Single process; the Adam moments live in the model; checkpoints are
// <exp>_epoch_N.cadckpt / final_model.cadckpt (named parameters and buffers, reference layout).
class GeometryTrainer {
public:
    using Config = TensorBoardTrainerEnhanced::Config;
    GeometryTrainer(std::shared_ptr<GeometryAwareNetworkImpl> model, std::shared_ptr<CombinedDepthLoss> loss_fn,
                    const Config& config)
        : model_(std::move(model)), loss_fn_(std::move(loss_fn)), config_(config) {
        if (!model_ || !loss_fn_) throw std::runtime_error("GeometryTrainer: model and loss are required");
        std::filesystem::create_directories(config_.checkpoint_dir);
        std::filesystem::create_directories(config_.log_dir);
        log_.open(config_.log_dir + "/training.log", std::ios::app);
        metrics_csv_.open(config_.log_dir + "/metrics.csv", std::ios::app);
        if (metrics_csv_.tellp() == 0)
            metrics_csv_ << "epoch,step,train_loss,val_loss,abs_rel,sq_rel,rmse,rmse_log,a1,a2,a3,learning_rate,time_elapsed\n";
    }

    void train(std::shared_ptr<SunRGBDLoader> train_loader, std::shared_ptr<SunRGBDLoader> val_loader = nullptr) {
        if (!train_loader) throw std::runtime_error("train: no training loader");
        const int B = config_.batch_size;
        const int nb = (int)(((int64_t)train_loader->size() + B - 1) / B);
        if (nb < 1) throw std::runtime_error("no training samples");
        msg("=== Starting Training (MI355X, geometry-aware network) ===");
        msg("Train samples: " + std::to_string(train_loader->size()) + ", batch size " + std::to_string(B) +
            ", epochs " + std::to_string(config_.num_epochs));
        const auto t0 = std::chrono::steady_clock::now();
        int64_t step = 0;
        for (int epoch = 1; epoch <= config_.num_epochs; ++epoch) {
            std::cout << "\n" << std::string(60, '=') << "\nEpoch " << epoch << "/" << config_.num_epochs << "\n";
            const float tl = trainEpoch(*train_loader, nb, step);
            TensorBoardTrainerEnhanced::ValidationMetrics vm;
            if (val_loader && config_.val_interval > 0 && epoch % config_.val_interval == 0) vm = validate(*val_loader);
            if (config_.save_interval > 0 && epoch % config_.save_interval == 0)
                save(config_.checkpoint_dir + "/" + config_.experiment_name + "_epoch_" + std::to_string(epoch) +
                     ".cadckpt");
            const long el = (long)std::chrono::duration_cast<std::chrono::seconds>(std::chrono::steady_clock::now() - t0).count();
            std::stringstream ss;
            ss << "Epoch " << epoch << " | Train Loss: " << std::fixed << std::setprecision(4) << tl;
            if (vm.loss > 0) ss << " | Val Loss: " << vm.loss << " | abs_rel: " << vm.abs_rel << " | rmse: " << vm.rmse;
            msg(ss.str());
            metrics_csv_ << epoch << "," << step << "," << tl << "," << vm.loss << "," << vm.abs_rel << "," << vm.sq_rel
                         << "," << vm.rmse << "," << vm.rmse_log << "," << vm.a1 << "," << vm.a2 << "," << vm.a3 << ","
                         << config_.learning_rate << "," << el << "\n";
            metrics_csv_.flush();
            step += nb;
        }
        save(config_.checkpoint_dir + "/final_model.cadckpt");
        msg("=== Training Complete ===");
    }

    // named parameters and buffers in the .cadckpt layout (no optimizer section)
    void save(const std::string& path) {
        std::ofstream f(path, std::ios::binary);
        if (!f) throw std::runtime_error("cannot write checkpoint " + path);
        auto ts = model_->named_parameters();
        auto bs = model_->named_buffers();
        ts.insert(ts.end(), bs.begin(), bs.end());
        f.write("CADCKPT1", 8);
        const int32_t n = (int32_t)ts.size();
        f.write((const char*)&n, 4);
        for (auto& t : ts) {
            const int32_t ln = (int32_t)t.name.size(), nd = (int32_t)t.shape.size();
            f.write((const char*)&ln, 4);
            f.write(t.name.data(), ln);
            f.write((const char*)&nd, 4);
            f.write((const char*)t.shape.data(), 8 * nd);
            f.write((const char*)t.value.data(), 4 * (int64_t)t.value.size());
        }
        msg("Checkpoint saved: " + path);
    }

private:
    void ensure(const SunRGBDLoader& L) {
        const int B = config_.batch_size, H = L.target_height(), W = L.target_width(), d = config_.device;
        if (rgb_.numel() == (int64_t)B * 3 * H * W) return;
        rgb_ = DeviceTensor::empty({B, 3, H, W}, d);
        gt_ = DeviceTensor::empty({B, 1, H, W}, d);
        K_ = DeviceTensor::empty({B, 3, 3}, d);
        rays_ = DeviceTensor::empty({B, 3, H, W}, d);
        cam_ = DeviceTensor::empty({B, 4}, d);
    }
    int next(cad_loader* ring) {
        const int n = cad_loader_next(ring, rgb_.data, gt_.data, K_.data, nullptr);
        if (n < 0) throw std::runtime_error(std::string("data loader: ") + cad_last_error());
        for (DeviceTensor* t : {&rgb_, &gt_, &K_, &rays_, &cam_}) t->shape[0] = n;
        const int H = (int)rgb_.size(2), W = (int)rgb_.size(3);
        cad::check(cad_ray_directions(K_.data, n, H, W, rays_.data, nullptr), "rays");   // a18
        cad::check(cad_camera_from_K(K_.data, n, cam_.data, nullptr), "camera_from_K");  // a15
        return n;
    }
    float trainEpoch(SunRGBDLoader& L, int nb, int64_t step0) {
        ensure(L);
        model_->train();
        cad_loader* ring = L.ring(config_.batch_size, config_.device, true);
        cad::check(cad_loader_start_epoch(ring, nullptr, (int64_t)L.size()), "start epoch");
        double total = 0.0;
        int64_t seen = 0;
        for (int bi = 0; bi < nb; ++bi) {
            const int n = next(ring);
            DeviceTensor pred = model_->forward(rgb_, rays_, cam_);
            DeviceTensor l = loss_fn_->forwardWithIntrinsics(pred, gt_, rgb_, K_);
            model_->backward(loss_fn_->dpred());
            model_->clip_grad_norm_(config_.use_grad_clip ? config_.grad_clip_value : INFINITY);
            model_->adam_step(config_.learning_rate, config_.weight_decay);
            const float lv = l.to_host()[0];
            if (!std::isfinite(lv)) throw std::runtime_error("non-finite loss at step " + std::to_string(step0 + bi));
            total += (double)lv * n;
            seen += n;
            if ((bi + 1) % std::max(1, config_.log_interval) == 0 || bi == nb - 1)
                std::cout << "\r  [" << std::setw(3) << (100 * (bi + 1) / nb) << "%] Batch " << (bi + 1) << "/" << nb
                          << " | Loss: " << std::fixed << std::setprecision(4) << lv << std::flush;
        }
        std::cout << std::endl;
        return (float)(total / std::max<int64_t>(1, seen));
    }
    TensorBoardTrainerEnhanced::ValidationMetrics validate(SunRGBDLoader& L) {
        ensure(L);
        model_->eval();
        TensorBoardTrainerEnhanced::ValidationMetrics m;
        const int64_t ns = std::min<int64_t>(500, (int64_t)L.size());
        cad_loader* ring = L.ring(1, config_.device, false);
        cad::check(cad_loader_start_epoch(ring, nullptr, ns), "validation");
        int count = 0;
        for (int64_t i = 0; i < ns; ++i) {
            next(ring);
            DeviceTensor pred = model_->forward(rgb_, rays_, cam_);
            DeviceTensor l = loss_fn_->forwardWithIntrinsics(pred, gt_, rgb_, K_);
            const DepthMetrics s = computeDepthMetrics(pred, gt_);
            m.loss += l.to_host()[0];
            m.abs_rel += s.abs_rel; m.sq_rel += s.sq_rel; m.rmse += s.rmse; m.rmse_log += s.rmse_log;
            m.a1 += s.a1; m.a2 += s.a2; m.a3 += s.a3;
            ++count;
        }
        if (count)
            for (float* p : {&m.loss, &m.abs_rel, &m.sq_rel, &m.rmse, &m.rmse_log, &m.a1, &m.a2, &m.a3}) *p /= count;
        model_->train();
        return m;
    }
    void msg(const std::string& s) {
        std::cout << s << std::endl;
        if (log_.is_open()) { log_ << s << "\n"; log_.flush(); }
    }

    std::shared_ptr<GeometryAwareNetworkImpl> model_;
    std::shared_ptr<CombinedDepthLoss> loss_fn_;
    Config config_;
    std::ofstream log_, metrics_csv_;
    DeviceTensor rgb_, gt_, K_, rays_, cam_;
};

}  // namespace camera_aware_depth

#endif  // CAD_TRAINER_HPP

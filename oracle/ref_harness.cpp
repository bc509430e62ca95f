// ORACLE / TEST INFRASTRUCTURE ONLY — never linked into or called by the product path.
//
// ref_harness: drives the REFERENCE implementation (header-only LibTorch code under
// /root/reference/src, compiled in place by oracle/Makefile against the pip LibTorch) through
// exactly the training step of TensorBoardTrainerEnhanced::trainEpoch
// (/root/reference/src/training/tensorboard_trainer_enhanced.h:287-304):
//     zero_grad -> BaselineUNetImpl::forward -> CombinedDepthLoss::forwardWithIntrinsics
//     -> backward -> clip_grad_norm_(params, 1.0) -> Adam::step  (Adam built as at :97-101)
// and dumps golden fixtures (mode "golden") or times the step on the host cores (mode "time",
// used by bench.py's cpu_baseline leg with kind="reference").
//
// --model selects the network:
//   baseline  BaselineUNetImpl(3, f, 10)                       models/baseline_unet.h:144-206
//   film      IntrinsicsConditionedUNetImpl(3, f, 4, 10)        models/intrinsics_unet.h:137-270
//             fed (B,4) [fx, fy, cx, cy] = [K00, K11, K02, K12] (a15: no reference code exists)
//   rayfilm   the config-3 composite of SURVEY §8 "Recommended config-3 model": enc1 =
//             RayEnhancedConv(3, f, 4, true) (geometry_aware_network.h:17-65) fed cat(rgb, rays),
//             enc2..dec1 = FiLMEncoderBlock / FiLMDecoderBlock (intrinsics_unet.h:59-113).
//   geo       GeometryAwareNetworkImpl(3, f, 4, 10, true, true)  models/geometry_aware_network.h:201-347
//             (RayEnhancedConv + CBAM encoders, ConvT + PCL + CBAM decoders, 6 levels) fed
//             (rgb, rays, (B,4) [fx, fy, cx, cy])
//   geolite   LightweightGeometryNetworkImpl(3, f, 4, 10)          geometry_aware_network.h:355-440
//
// Inputs are the synthetic SUN-RGB-D-shaped batches of SURVEY.md §8(d): a counter-based
// splitmix64 stream so that every consumer (this harness, oracle/cad_oracle.py, bench.py) can
// regenerate identical bytes.  Outputs: <out>/manifest.json + <out>/tensors.bin (raw f32 LE).
#include <torch/torch.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "models/baseline_unet.h"
#include "models/geometry_aware_network.h"
#include "models/intrinsics_unet.h"
#include "loss/depth_loss.h"

using namespace camera_aware_depth;

namespace {

uint64_t splitmix64(uint64_t seed, uint64_t idx) {
    uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
float u01(uint64_t seed, uint64_t idx) {
    uint32_t u = (uint32_t)(splitmix64(seed, idx) >> 32);
    return (float)(u >> 8) * (1.0f / 16777216.0f);
}

struct Batch { torch::Tensor rgb, gt, K, cam4, rays; };

// SURVEY.md §8(d) synthetic batch (rgb U[0,1), smooth depth with Kinect-style holes, per-sample K).
Batch make_batch(int B, int H, int W, uint64_t rgb_seed = 0xC0FFEE, uint64_t hole_seed = 0xD3E7) {
    Batch b;
    b.rgb = torch::empty({B, 3, H, W});
    b.gt = torch::empty({B, 1, H, W});
    b.K = torch::zeros({B, 3, 3});
    float* r = b.rgb.data_ptr<float>();
    for (int64_t i = 0; i < (int64_t)B * 3 * H * W; ++i) r[i] = u01(rgb_seed, i);
    float* g = b.gt.data_ptr<float>();
    for (int bb = 0; bb < B; ++bb)
        for (int v = 0; v < H; ++v)
            for (int u = 0; u < W; ++u) {
                int64_t idx = ((int64_t)bb * H + v) * W + u;
                double ph = 2.0 * M_PI * ((double)u / W * 1.3 + (double)v / H * 0.7 + 0.1 * bb);
                double d = 0.5 + 9.0 * (0.5 + 0.5 * std::sin(ph));
                d = std::min(9.5, std::max(0.5, d));
                if (u01(hole_seed, idx) < 0.15f || v < H / 16) d = 0.0;
                g[idx] = (float)d;
            }
    float* k = b.K.data_ptr<float>();
    for (int bb = 0; bb < B; ++bb) {
        float fx, fy, cx, cy;
        if (bb % 2 == 0) { fx = 518.858f; fy = 519.470f; cx = 325.582f; cy = 253.736f; }
        else { fx = 570.342f; fy = 570.342f; cx = 320.0f; cy = 240.0f; }
        float sx = (float)W / 640.0f, sy = (float)H / 480.0f;   // sunrgbd_loader.cpp:480-488
        float* kk = k + bb * 9;
        kk[0] = fx * sx; kk[2] = cx * sx; kk[4] = fy * sy; kk[5] = cy * sy; kk[8] = 1.0f;
    }
    // a15: (B,3,3) -> (B,4) [fx, fy, cx, cy]
    b.cam4 = torch::stack({b.K.select(1, 0).select(1, 0), b.K.select(1, 1).select(1, 1),
                           b.K.select(1, 0).select(1, 2), b.K.select(1, 1).select(1, 2)}, 1).contiguous();
    // a18: RayDirectionComputer::computeRayDirections (ray_direction_computer.cpp:17-62) restated
    // (that .cpp needs Eigen, absent here), laid out (B,3,H,W) as the loader reshapes it
    // (sunrgbd_loader.cpp:346-347), computed directly at the working resolution from the scaled K.
    b.rays = torch::empty({B, 3, H, W});
    float* ry = b.rays.data_ptr<float>();
    for (int bb = 0; bb < B; ++bb) {
        const float* kk = k + bb * 9;
        const float fx_inv = 1.0f / kk[0], fy_inv = 1.0f / kk[4], cx = kk[2], cy = kk[5];
        for (int v = 0; v < H; ++v)
            for (int u = 0; u < W; ++u) {
                const float x = ((float)u - cx) * fx_inv, y = ((float)v - cy) * fy_inv, z = 1.0f;
                const float n = std::sqrt(x * x + y * y + z * z);
                const int64_t o = (int64_t)v * W + u, hw = (int64_t)H * W;
                ry[((int64_t)bb * 3 + 0) * hw + o] = x / n;
                ry[((int64_t)bb * 3 + 1) * hw + o] = y / n;
                ry[((int64_t)bb * 3 + 2) * hw + o] = z / n;
            }
    }
    return b;
}

// IntrinsicsConditionedUNetImpl::normalizeCameraIntrinsics (intrinsics_unet.h:252-268) is private;
// the composite below needs the same (B,4) normalisation (a14), so it is restated with the same ops.
torch::Tensor normalize_cam(torch::Tensor in, int width, int height) {
    using torch::indexing::Slice;
    auto n = in.clone();
    n.index_put_({Slice(), 0}, in.index({Slice(), 0}) / width);
    n.index_put_({Slice(), 1}, in.index({Slice(), 1}) / height);
    n.index_put_({Slice(), 2}, (in.index({Slice(), 2}) / width) * 2.0f - 1.0f);
    n.index_put_({Slice(), 3}, (in.index({Slice(), 3}) / height) * 2.0f - 1.0f);
    return n;
}

// Config-3 composite from reference classes only (no new math): module registration order equals
// IntrinsicsConditionedUNetImpl's, so parameter names match it (enc1.* is a RayEnhancedConv whose
// conv1 takes 3 + 3 ray channels).  32,862,465 parameters at f = 64.
struct RayFiLMUNetImpl : torch::nn::Module {
    RayEnhancedConv enc1{nullptr};
    FiLMEncoderBlock enc2{nullptr}, enc3{nullptr}, enc4{nullptr}, bottleneck{nullptr};
    FiLMDecoderBlock dec4{nullptr}, dec3{nullptr}, dec2{nullptr}, dec1{nullptr};
    torch::nn::Conv2d out_conv{nullptr};
    float max_depth;
    RayFiLMUNetImpl(int f, float md) : max_depth(md) {
        enc1 = register_module("enc1", RayEnhancedConv(3, f, 4, true));
        enc2 = register_module("enc2", FiLMEncoderBlock(f, f * 2, 4));
        enc3 = register_module("enc3", FiLMEncoderBlock(f * 2, f * 4, 4));
        enc4 = register_module("enc4", FiLMEncoderBlock(f * 4, f * 8, 4));
        bottleneck = register_module("bottleneck", FiLMEncoderBlock(f * 8, f * 16, 4));
        dec4 = register_module("dec4", FiLMDecoderBlock(f * 16, f * 8, 4));
        dec3 = register_module("dec3", FiLMDecoderBlock(f * 8, f * 4, 4));
        dec2 = register_module("dec2", FiLMDecoderBlock(f * 4, f * 2, 4));
        dec1 = register_module("dec1", FiLMDecoderBlock(f * 2, f, 4));
        out_conv = register_module("out_conv", torch::nn::Conv2d(torch::nn::Conv2dOptions(f, 1, 1)));
    }
    torch::Tensor forward(torch::Tensor x, torch::Tensor cam4, torch::Tensor rays) {
        auto c = normalize_cam(cam4, x.size(3), x.size(2));
        auto s1 = enc1(x, c, rays);
        auto s2 = enc2(s1, c);
        auto s3 = enc3(s2, c);
        auto s4 = enc4(s3, c);
        auto y = bottleneck(s4, c);
        y = dec4(y, s4, c);
        y = dec3(y, s3, c);
        y = dec2(y, s2, c);
        y = dec1(y, s1, c);
        return torch::sigmoid(out_conv(y)) * max_depth;
    }
};
TORCH_MODULE(RayFiLMUNet);

// --init synth: every parameter (named_parameters() order, running element offset `off`) is set from
// the counter stream so fixtures need not store initial weights (tests regenerate them with
// oracle/cad_oracle.py:synth_init, bit-identically):
//   u = u01(0x1A17, off + i);  dim >= 2: (2u - 1) / sqrt(numel / size(0))
//   1-D *.weight (BN affine) and *.fc_gamma.bias: 1 + 0.1 (2u - 1);  other 1-D: 0.1 (2u - 1)
void synth_init(torch::nn::Module& m) {
    torch::NoGradGuard ng;
    int64_t off = 0;
    for (auto& kv : m.named_parameters()) {
        auto t = kv.value();
        const std::string& n = kv.key();
        auto ends = [&](const std::string& suf) {
            return n.size() >= suf.size() && n.compare(n.size() - suf.size(), suf.size(), suf) == 0;
        };
        auto c = torch::empty_like(t).contiguous();
        float* p = c.data_ptr<float>();
        const int64_t N = c.numel();
        const float bound = t.dim() >= 2 ? 1.0f / std::sqrt((float)(N / t.size(0))) : 0.f;
        const bool one = t.dim() == 1 && (ends(".weight") || ends(".fc_gamma.bias"));
        for (int64_t i = 0; i < N; ++i) {
            const float u = u01(0x1A17, off + i);
            p[i] = t.dim() >= 2 ? (2.0f * u - 1.0f) * bound : one ? 1.0f + 0.1f * (2.0f * u - 1.0f) : 0.1f * (2.0f * u - 1.0f);
        }
        t.copy_(c);
        off += N;
    }
}

// one network of --model behind a common face
struct Net {
    std::shared_ptr<torch::nn::Module> mod;
    std::function<torch::Tensor(const Batch&)> fwd;
    int64_t count() const {
        int64_t n = 0;
        for (auto& p : mod->parameters()) n += p.numel();
        return n;
    }
};

Net make_net(const std::string& kind, int f) {
    Net n;
    if (kind == "baseline") {
        auto m = std::make_shared<BaselineUNetImpl>(3, f, 10.0f);   // train_main.cpp:325-333
        n.mod = m;
        n.fwd = [m](const Batch& b) { return m->forward(b.rgb); };
    } else if (kind == "film") {
        auto m = std::make_shared<IntrinsicsConditionedUNetImpl>(3, f, 4, 10.0f);
        n.mod = m;
        n.fwd = [m](const Batch& b) { return m->forward(b.rgb, b.cam4); };
    } else if (kind == "rayfilm") {
        auto m = std::make_shared<RayFiLMUNetImpl>(f, 10.0f);
        n.mod = m;
        n.fwd = [m](const Batch& b) { return m->forward(b.rgb, b.cam4, b.rays); };
    } else if (kind == "geo") {
        auto m = std::make_shared<GeometryAwareNetworkImpl>(3, f, 4, 10.0f, true, true);
        n.mod = m;
        n.fwd = [m](const Batch& b) { return m->forward(b.rgb, b.rays, b.cam4); };
    } else if (kind == "geolite") {
        auto m = std::make_shared<LightweightGeometryNetworkImpl>(3, f, 4, 10.0f);
        n.mod = m;
        n.fwd = [m](const Batch& b) { return m->forward(b.rgb, b.rays, b.cam4); };
    } else {
        fprintf(stderr, "unknown --model %s\n", kind.c_str());
        exit(2);
    }
    return n;
}

struct Dumper {
    std::string dir;
    std::ofstream bin;
    std::ostringstream man;
    int64_t off = 0;
    bool first = true;
    explicit Dumper(const std::string& d) : dir(d), bin(d + "/tensors.bin", std::ios::binary) {
        man << "{\n \"tensors\": [\n";
    }
    void add(const std::string& name, torch::Tensor t) {
        t = t.detach().to(torch::kFloat32).contiguous();
        bin.write((const char*)t.data_ptr<float>(), t.numel() * 4);
        if (!first) man << ",\n";
        first = false;
        man << "  {\"name\": \"" << name << "\", \"offset\": " << off << ", \"shape\": [";
        for (int i = 0; i < t.dim(); ++i) man << (i ? ", " : "") << t.size(i);
        man << "]}";
        off += t.numel();
    }
    void finish(const std::string& meta) {
        man << "\n ],\n \"meta\": " << meta << "\n}\n";
        std::ofstream(dir + "/manifest.json") << man.str();
    }
};

// a20: TensorBoardTrainerEnhanced::computeDepthMetrics (tensorboard_trainer_enhanced.h:400-439);
// that header cannot be compiled here (it pulls the OpenCV loader / TB logger), so the ~20 lines of
// metric math are restated with the same ATen ops.  Returns abs_rel averaged per sample.
double abs_rel_per_sample(torch::Tensor pred, torch::Tensor gt) {
    double acc = 0.0;
    for (int b = 0; b < pred.size(0); ++b) {
        auto p = pred[b].view({-1}), g = gt[b].view({-1});
        auto m = g > 0.0f;
        auto pv = p.masked_select(m), gv = g.masked_select(m);
        if (pv.numel() == 0) continue;
        acc += (torch::abs(pv - gv) / gv).mean().item<float>();
    }
    return acc / pred.size(0);
}

struct Args {
    std::string mode = "golden", out = ".", model = "baseline", init = "default", ckpt;
    int f = 8, B = 2, H = 64, W = 64, steps = 3, threads = 1, warmup = 1, holes_all = 0, mask_seed = 0, lean = 0;
    float w[4] = {1.0f, 0.1f, 0.001f, 0.01f};
    float lr = 1e-4f, wd = 1e-5f, clip = 1.0f;
};

Args parse(int argc, char** argv) {
    Args a;
    for (int i = 1; i + 1 < argc; i += 2) {
        std::string k = argv[i], v = argv[i + 1];
        if (k == "--mode") a.mode = v;
        else if (k == "--out") a.out = v;
        else if (k == "--ckpt") a.ckpt = v;
        else if (k == "--model") a.model = v;
        else if (k == "--init") a.init = v;
        else if (k == "--f") a.f = std::stoi(v);
        else if (k == "--B") a.B = std::stoi(v);
        else if (k == "--H") a.H = std::stoi(v);
        else if (k == "--W") a.W = std::stoi(v);
        else if (k == "--steps") a.steps = std::stoi(v);
        else if (k == "--warmup") a.warmup = std::stoi(v);
        else if (k == "--threads") a.threads = std::stoi(v);
        else if (k == "--weights") sscanf(v.c_str(), "%f,%f,%f,%f", &a.w[0], &a.w[1], &a.w[2], &a.w[3]);
        else if (k == "--lr") a.lr = std::stof(v);
        else if (k == "--wd") a.wd = std::stof(v);
        else if (k == "--holes-all") a.holes_all = std::stoi(v);
        else if (k == "--mask-seed") a.mask_seed = std::stoi(v);
        else if (k == "--lean") a.lean = std::stoi(v);   // golden: no final.param.* (large models)
        else { fprintf(stderr, "unknown arg %s\n", k.c_str()); exit(2); }
    }
    return a;
}

}  // namespace

int main(int argc, char** argv) {
    Args a = parse(argc, argv);
    torch::set_num_threads(a.threads);
    torch::manual_seed(42);   // train_main.cpp:318 -> setupSeeds(42)

    Net net = make_net(a.model, a.f);
    auto& model = net.mod;
    const bool synth = a.init == "synth";
    if (synth) synth_init(*model);
    CombinedDepthLoss loss_fn(a.w[0], a.w[1], a.w[2], a.w[3]);        // train_main.cpp:352-357
    torch::optim::Adam opt(model->parameters(),
                           torch::optim::AdamOptions(a.lr).weight_decay(a.wd));   // enhanced.h:97-101
    Batch batch = make_batch(a.B, a.H, a.W);

    auto step = [&](torch::Tensor* pred_out, torch::Tensor* dpred_out, double* norm_out,
                    std::vector<torch::Tensor>* grads_pre_clip) -> float {
        model->train();
        opt.zero_grad();
        auto pred = net.fwd(batch);
        if (dpred_out) pred.retain_grad();
        auto loss = loss_fn.forwardWithIntrinsics(pred, batch.gt, batch.rgb, batch.K);
        loss.backward();
        if (grads_pre_clip)
            for (auto& p : model->parameters()) grads_pre_clip->push_back(p.grad().clone());
        double n = torch::nn::utils::clip_grad_norm_(model->parameters(), a.clip);
        opt.step();
        if (pred_out) *pred_out = pred.detach().clone();
        if (dpred_out) *dpred_out = pred.grad().clone();
        if (norm_out) *norm_out = n;
        return loss.item<float>();
    };

    if (a.mode == "time") {
        for (int i = 0; i < a.warmup; ++i) step(nullptr, nullptr, nullptr, nullptr);
        auto t0 = std::chrono::steady_clock::now();
        float last = 0;
        for (int i = 0; i < a.steps; ++i) last = step(nullptr, nullptr, nullptr, nullptr);
        double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        printf("{\"images_per_s\": %.6f, \"seconds\": %.3f, \"steps\": %d, \"batch\": %d, \"H\": %d, "
               "\"W\": %d, \"f\": %d, \"threads\": %d, \"last_loss\": %.6f, \"model\": \"%s\"}\n",
               a.steps * a.B / s, s, a.steps, a.B, a.H, a.W, a.f, a.threads, last, a.model.c_str());
        return 0;
    }

    if (a.mode == "save" || a.mode == "load") {
        // Checkpoint compatibility: "save" trains --steps steps (so the BN running statistics and
        // num_batches_tracked are not the defaults) and writes the reference's checkpoint,
        // torch::save(model_, path) (tensorboard_trainer_enhanced.h:656-662); "load" reads a
        // checkpoint into a fresh --model with torch::load(model, path) — the archive reader a
        // reference user resumes or evaluates with.  Both dump every named parameter and buffer.
        if (a.mode == "load") torch::load(model, a.ckpt);
        else {
            for (int i = 0; i < a.steps; ++i) step(nullptr, nullptr, nullptr, nullptr);
            torch::save(model, a.ckpt);
        }
        Dumper d(a.out);
        for (auto& kv : model->named_parameters()) d.add("param." + kv.key(), kv.value());
        for (auto& kv : model->named_buffers()) d.add("buffer." + kv.key(), kv.value());
        std::ostringstream meta;
        meta << "{\"model\": \"" << a.model << "\", \"f\": " << a.f << ", \"mode\": \"" << a.mode << "\", \"steps\": " << a.steps << "}";
        d.finish(meta.str());
        printf("%s %s\n", a.mode.c_str(), a.ckpt.c_str());
        return 0;
    }

    if (a.mode == "loss") {
        // Loss-only golden: pred = 0.05 + 9.9*U[0,1) (seed 0xBEEF), gt/rgb/K from make_batch;
        // --holes-all makes every gt pixel invalid (the n == 0 branches of depth_loss.h:53,325).
        // --mask-seed S passes forwardWithIntrinsics' optional valid_mask (:416-433): u01(S, i) < 0.8,
        // independent of gt (so it also admits gt == 0 pixels, and drops valid ones).
        auto pred = torch::empty({a.B, 1, a.H, a.W});
        float* pp = pred.data_ptr<float>();
        for (int64_t i = 0; i < pred.numel(); ++i) pp[i] = 0.05f + 9.9f * u01(0xBEEF, i);
        if (a.holes_all) batch.gt.zero_();
        torch::optional<torch::Tensor> mask = torch::nullopt;
        torch::Tensor maskf;
        if (a.mask_seed) {
            maskf = torch::empty({a.B, 1, a.H, a.W});
            float* mp = maskf.data_ptr<float>();
            for (int64_t i = 0; i < maskf.numel(); ++i) mp[i] = u01((uint64_t)a.mask_seed, i) < 0.8f ? 1.f : 0.f;
            mask = maskf > 0.5f;
        }
        pred.requires_grad_(true);
        auto total = loss_fn.forwardWithIntrinsics(pred, batch.gt, batch.rgb, batch.K, mask);
        total.backward();
        torch::NoGradGuard ng;
        auto comps = loss_fn.getComponentsWithIntrinsics(pred.detach(), batch.gt, batch.rgb, batch.K, mask);
        Dumper d(a.out);
        d.add("input.pred", pred);
        d.add("input.gt", batch.gt);
        if (a.mask_seed) d.add("input.mask", maskf);
        d.add("dpred", pred.grad());
        std::ostringstream meta;
        meta.precision(9);
        meta << "{\"B\": " << a.B << ", \"H\": " << a.H << ", \"W\": " << a.W << ", \"weights\": ["
             << a.w[0] << ", " << a.w[1] << ", " << a.w[2] << ", " << a.w[3] << "], \"holes_all\": "
             << a.holes_all << ", \"mask_seed\": " << a.mask_seed << ", \"total\": " << total.item<float>() << ", \"total_dim\": " << total.dim()
             << ", \"components\": {";
        bool first = true;
        for (auto& kv : comps) { meta << (first ? "" : ", ") << "\"" << kv.first << "\": " << kv.second; first = false; }
        meta << "}}";
        d.finish(meta.str());
        printf("wrote %s (loss=%.6f)\n", a.out.c_str(), total.item<float>());
        return 0;
    }

    Dumper d(a.out);
    d.add("input.rgb", batch.rgb);
    d.add("input.gt", batch.gt);
    d.add("input.K", batch.K);
    if (a.model != "baseline") d.add("input.cam4", batch.cam4);
    if (a.model == "rayfilm" || a.model == "geo" || a.model == "geolite") d.add("input.rays", batch.rays);
    if (!synth) {   // synth init: regenerated by the tests, buffers are the module defaults
        for (auto& kv : model->named_parameters()) d.add("init." + kv.key(), kv.value());
        for (auto& kv : model->named_buffers())
            if (kv.value().is_floating_point()) d.add("init." + kv.key(), kv.value());
    }

    torch::Tensor pred1, dpred1;
    double norm1 = 0;
    std::vector<torch::Tensor> g1;
    std::map<std::string, float> comps1;
    std::vector<float> losses;
    losses.push_back(step(&pred1, &dpred1, &norm1, &g1));
    {
        torch::NoGradGuard ng;
        comps1 = loss_fn.getComponentsWithIntrinsics(pred1, batch.gt, batch.rgb, batch.K);
    }
    d.add("step1.pred", pred1);
    d.add("step1.dpred", dpred1);
    {
        auto names = model->named_parameters();
        int i = 0;
        for (auto& kv : names) d.add("step1.grad." + kv.key(), g1[i++]);
        if (!synth)
            for (auto& kv : names) d.add("step1.param." + kv.key(), kv.value());
        for (auto& kv : model->named_buffers())
            if (kv.value().is_floating_point()) d.add("step1." + kv.key(), kv.value());
    }
    for (int s = 1; s < a.steps; ++s) losses.push_back(step(nullptr, nullptr, nullptr, nullptr));
    if (!a.lean)
        for (auto& kv : model->named_parameters()) d.add("final.param." + kv.key(), kv.value());
    for (auto& kv : model->named_buffers())
        if (kv.value().is_floating_point()) d.add("final." + kv.key(), kv.value());
    // eval-mode forward after training (BN running statistics) + a20 abs_rel
    torch::Tensor pred_eval;
    {
        torch::NoGradGuard ng;
        model->eval();
        pred_eval = net.fwd(batch);
    }
    d.add("final.pred_eval", pred_eval);
    double absrel = abs_rel_per_sample(pred_eval, batch.gt);

    std::ostringstream meta;
    meta.precision(9);
    meta << "{\"model\": \"" << a.model << "\", \"init\": \"" << a.init << "\", \"f\": " << a.f << ", \"B\": " << a.B << ", \"H\": " << a.H << ", \"W\": " << a.W
         << ", \"steps\": " << a.steps << ", \"threads\": " << a.threads
         << ", \"weights\": [" << a.w[0] << ", " << a.w[1] << ", " << a.w[2] << ", " << a.w[3] << "]"
         << ", \"lr\": " << a.lr << ", \"wd\": " << a.wd << ", \"clip\": " << a.clip
         << ", \"num_params\": " << net.count()
         << ", \"step1_total_norm\": " << norm1 << ", \"losses\": [";
    for (size_t i = 0; i < losses.size(); ++i) meta << (i ? ", " : "") << losses[i];
    meta << "], \"step1_components\": {";
    bool first = true;
    for (auto& kv : comps1) { meta << (first ? "" : ", ") << "\"" << kv.first << "\": " << kv.second; first = false; }
    meta << "}, \"final_abs_rel_eval\": " << absrel << "}";
    d.finish(meta.str());
    printf("wrote %s (num_params=%lld, loss1=%.6f)\n", a.out.c_str(), (long long)net.count(), losses[0]);
    return 0;
}

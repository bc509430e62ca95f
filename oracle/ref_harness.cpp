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
// Inputs are the synthetic SUN-RGB-D-shaped batches of SURVEY.md §8(d): a counter-based
// splitmix64 stream so that every consumer (this harness, oracle/cad_oracle.py, bench.py) can
// regenerate identical bytes.  Outputs: <out>/manifest.json + <out>/tensors.bin (raw f32 LE).
#include <torch/torch.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "models/baseline_unet.h"
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

struct Batch { torch::Tensor rgb, gt, K; };

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
    return b;
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
    std::string mode = "golden", out = ".";
    int f = 8, B = 2, H = 64, W = 64, steps = 3, threads = 1, warmup = 1, holes_all = 0;
    float w[4] = {1.0f, 0.1f, 0.001f, 0.01f};
    float lr = 1e-4f, wd = 1e-5f, clip = 1.0f;
};

Args parse(int argc, char** argv) {
    Args a;
    for (int i = 1; i + 1 < argc; i += 2) {
        std::string k = argv[i], v = argv[i + 1];
        if (k == "--mode") a.mode = v;
        else if (k == "--out") a.out = v;
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
        else { fprintf(stderr, "unknown arg %s\n", k.c_str()); exit(2); }
    }
    return a;
}

}  // namespace

int main(int argc, char** argv) {
    Args a = parse(argc, argv);
    torch::set_num_threads(a.threads);
    torch::manual_seed(42);   // train_main.cpp:318 -> setupSeeds(42)

    auto model = std::make_shared<BaselineUNetImpl>(3, a.f, 10.0f);   // train_main.cpp:325-333
    CombinedDepthLoss loss_fn(a.w[0], a.w[1], a.w[2], a.w[3]);        // train_main.cpp:352-357
    torch::optim::Adam opt(model->parameters(),
                           torch::optim::AdamOptions(a.lr).weight_decay(a.wd));   // enhanced.h:97-101
    Batch batch = make_batch(a.B, a.H, a.W);

    auto step = [&](torch::Tensor* pred_out, torch::Tensor* dpred_out, double* norm_out,
                    std::vector<torch::Tensor>* grads_pre_clip) -> float {
        model->train();
        opt.zero_grad();
        auto pred = model->forward(batch.rgb);
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
               "\"W\": %d, \"f\": %d, \"threads\": %d, \"last_loss\": %.6f}\n",
               a.steps * a.B / s, s, a.steps, a.B, a.H, a.W, a.f, a.threads, last);
        return 0;
    }

    if (a.mode == "loss") {
        // Loss-only golden: pred = 0.05 + 9.9*U[0,1) (seed 0xBEEF), gt/rgb/K from make_batch;
        // --holes-all makes every gt pixel invalid (the n == 0 branches of depth_loss.h:53,325).
        auto pred = torch::empty({a.B, 1, a.H, a.W});
        float* pp = pred.data_ptr<float>();
        for (int64_t i = 0; i < pred.numel(); ++i) pp[i] = 0.05f + 9.9f * u01(0xBEEF, i);
        if (a.holes_all) batch.gt.zero_();
        pred.requires_grad_(true);
        auto total = loss_fn.forwardWithIntrinsics(pred, batch.gt, batch.rgb, batch.K);
        total.backward();
        torch::NoGradGuard ng;
        auto comps = loss_fn.getComponentsWithIntrinsics(pred.detach(), batch.gt, batch.rgb, batch.K);
        Dumper d(a.out);
        d.add("input.pred", pred);
        d.add("input.gt", batch.gt);
        d.add("dpred", pred.grad());
        std::ostringstream meta;
        meta.precision(9);
        meta << "{\"B\": " << a.B << ", \"H\": " << a.H << ", \"W\": " << a.W << ", \"weights\": ["
             << a.w[0] << ", " << a.w[1] << ", " << a.w[2] << ", " << a.w[3] << "], \"holes_all\": "
             << a.holes_all << ", \"total\": " << total.item<float>() << ", \"total_dim\": " << total.dim()
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
    for (auto& kv : model->named_parameters()) d.add("init." + kv.key(), kv.value());
    for (auto& kv : model->named_buffers())
        if (kv.value().is_floating_point()) d.add("init." + kv.key(), kv.value());

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
        for (auto& kv : names) d.add("step1.param." + kv.key(), kv.value());
        for (auto& kv : model->named_buffers())
            if (kv.value().is_floating_point()) d.add("step1." + kv.key(), kv.value());
    }
    for (int s = 1; s < a.steps; ++s) losses.push_back(step(nullptr, nullptr, nullptr, nullptr));
    for (auto& kv : model->named_parameters()) d.add("final.param." + kv.key(), kv.value());
    for (auto& kv : model->named_buffers())
        if (kv.value().is_floating_point()) d.add("final." + kv.key(), kv.value());
    // eval-mode forward after training (BN running statistics) + a20 abs_rel
    torch::Tensor pred_eval;
    {
        torch::NoGradGuard ng;
        model->eval();
        pred_eval = model->forward(batch.rgb);
    }
    d.add("final.pred_eval", pred_eval);
    double absrel = abs_rel_per_sample(pred_eval, batch.gt);

    std::ostringstream meta;
    meta.precision(9);
    meta << "{\"f\": " << a.f << ", \"B\": " << a.B << ", \"H\": " << a.H << ", \"W\": " << a.W
         << ", \"steps\": " << a.steps << ", \"threads\": " << a.threads
         << ", \"weights\": [" << a.w[0] << ", " << a.w[1] << ", " << a.w[2] << ", " << a.w[3] << "]"
         << ", \"lr\": " << a.lr << ", \"wd\": " << a.wd << ", \"clip\": " << a.clip
         << ", \"num_params\": " << model->count_parameters()
         << ", \"step1_total_norm\": " << norm1 << ", \"losses\": [";
    for (size_t i = 0; i < losses.size(); ++i) meta << (i ? ", " : "") << losses[i];
    meta << "], \"step1_components\": {";
    bool first = true;
    for (auto& kv : comps1) { meta << (first ? "" : ", ") << "\"" << kv.first << "\": " << kv.second; first = false; }
    meta << "}, \"final_abs_rel_eval\": " << absrel << "}";
    d.finish(meta.str());
    printf("wrote %s (num_params=%lld, loss1=%.6f)\n", a.out.c_str(), (long long)model->count_parameters(), losses[0]);
    return 0;
}

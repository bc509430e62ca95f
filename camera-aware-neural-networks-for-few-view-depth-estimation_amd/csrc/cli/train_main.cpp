// build/train — drop-in for the reference's `./build/train --config <yaml>` entry point
// (src/training/train_main.cpp:279-507 driving TensorBoardTrainerEnhanced, enhanced.h:142-334),
// on libcad_hip.so through the C++ drop-in classes of include/cad/cad.hpp.
//
//   build/train -c configs/train_config.yaml [-e baseline_unet] [-g 0] [-d] [--tensorboard true]
//               [-r checkpoint.cadckpt | model.pt]
//
// Same flags and defaults (train_main.cpp:38-45), same YAML keys (loadConfig :60-167, main :297-430),
// same per-batch step (enhanced.h:287-304), sample-weighted epoch loss (:308,333), validation every
// val_interval with computeDepthMetrics averaged per sample (:339-439), metrics.csv with the
// reference's header (:104-115), checkpoints every save_interval (:218-220).  Exit 0 on success;
// any exception prints "Error: <what>" and exits 1 (:503-506).
// Deliberate differences: the model lives on the GPU (the reference never moves it,
// SURVEY §0 fact 2); --resume really resumes (params + BN buffers + Adam state; the reference parses
// and ignores it); TensorBoard events are written as a CSV of scalars (no Python tensorboard here);
// the dataset is data.dataset_name: "synthetic" (SUN-RGB-D-shaped counter-based samples) — decoding
// the real SUN RGB-D JPEG/PNG files needs OpenCV, absent on this image.
#include <signal.h>
#include <spawn.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <iostream>
#include <algorithm>
#include <memory>
#include <random>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/cad/cad.hpp"
#include "../host/yaml_lite.hpp"

namespace fs = std::filesystem;
using namespace camera_aware_depth;

namespace {

struct Args {
    std::string config = "configs/train_config.yaml", experiment = "baseline_unet", resume;
    int gpu = 0;
    bool debug = false, tensorboard = true;
    bool dry_run = false;   // print the (per-rank) run plan and exit before any GPU call
    std::vector<std::string> argv;
};

void usage() {
    std::cout << "train - Train depth estimation models (MI355X)\n"
                 "  -c, --config arg      Path to config file (default: configs/train_config.yaml)\n"
                 "  -e, --experiment arg  Experiment name (default: baseline_unet)\n"
                 "  -r, --resume arg      Resume from checkpoint (.cadckpt: weights + optimizer;\n"
                 "                        .pt: torch::save model archive, weights only)\n"
                 "  -g, --gpu arg         GPU ID (default: 0)\n"
                 "  -d, --debug           Enable debug mode\n"
                 "      --tensorboard arg Enable TensorBoard-style scalar logging (default: true)\n"
                 "      --dry-run         Print the run plan (per data-parallel rank) and exit; no GPU use\n"
                 "  -h, --help            Print help\n";
}

Args parse_args(int argc, char** argv) {
    Args a;
    a.argv.assign(argv, argv + argc);
    for (int i = 1; i < argc; ++i) {
        std::string k = argv[i], v;
        auto eq = k.find('=');
        if (eq != std::string::npos) { v = k.substr(eq + 1); k = k.substr(0, eq); }
        auto next = [&]() -> std::string {
            if (!v.empty()) return v;
            if (i + 1 >= argc) throw std::runtime_error("missing value for " + k);
            return argv[++i];
        };
        if (k == "-h" || k == "--help") { usage(); std::exit(0); }
        else if (k == "-c" || k == "--config") a.config = next();
        else if (k == "-e" || k == "--experiment") a.experiment = next();
        else if (k == "-r" || k == "--resume") a.resume = next();
        else if (k == "-g" || k == "--gpu") a.gpu = std::stoi(next());
        else if (k == "-d" || k == "--debug") a.debug = v.empty() ? true : (v == "true" || v == "1");
        else if (k == "--dry-run") a.dry_run = true;
        else if (k == "--tensorboard") {
            std::string t = (!v.empty() || (i + 1 < argc && argv[i + 1][0] != '-')) ? next() : "true";
            a.tensorboard = t == "true" || t == "1";
        } else throw std::runtime_error("unknown option " + k);
    }
    return a;
}

struct Config {   // the TrainingConfig fields the step uses (trainer.h:24-92)
    int num_epochs = 50, batch_size = 8, log_interval = 10, val_interval = 1, save_interval = 5;
    float learning_rate = 1e-4f, weight_decay = 1e-5f, grad_clip_value = 1.0f;
    bool use_grad_clip = true;
    float si = 1.0f, grad = 0.1f, smooth = 0.001f, reproj = 0.01f, max_depth = 10.0f;
    int init_features = 64, height = 240, width = 320, seed = 42;
    std::string checkpoint_dir = "./checkpoints", log_dir = "./logs", experiment_name = "baseline_unet";
    std::string dataset = "sunrgbd";
    std::string manifest_path = "./data/sunrgbd_manifest.json";
    int n_train = 64, n_val = 16;
    // data.augmentation (train_main.cpp:377-386 -> AugmentationConfig, random_seed 42)
    bool aug_crop = true, aug_flip = true, aug_jitter = true;
    float aug_flip_p = 0.5f, aug_brightness = 0.2f, aug_contrast = 0.2f;
    // hardware: (configs/train_config.yaml:176-183; parsed but unused by the reference)
    bool distributed = false;
    int num_gpus = 1;
    std::vector<int> gpu_ids;
    std::string backend = "nccl";
};

Config load_config(const yaml_lite::Node& y, const std::string& experiment) {   // train_main.cpp:60-167
    Config c;
    c.experiment_name = experiment;
    if (auto& o = y["optimization"]) {
        c.learning_rate = o["learning_rate"].as<float>(1e-4f);
        c.weight_decay = o["weight_decay"].as<float>(1e-5f);
        if (o["gradient_clip"]) {
            c.use_grad_clip = o["gradient_clip"].as<bool>(true);
            c.grad_clip_value = o["gradient_clip_value"].as<float>(1.0f);
        }
    }
    if (auto& t = y["training"]) {
        c.num_epochs = t["num_epochs"].as<int>(50);
        c.batch_size = t["batch_size"].as<int>(8);
        c.log_interval = t["log_interval"].as<int>(10);
        c.val_interval = t["val_interval"].as<int>(1);
    }
    if (auto& l = y["loss"]) {
        c.si = l["si_weight"].as<float>(1.0f);
        c.grad = l["grad_weight"].as<float>(0.1f);
        c.smooth = l["smooth_weight"].as<float>(0.001f);
        c.reproj = l["reproj_weight"].as<float>(0.01f);
    }
    if (auto& k = y["checkpointing"]) {
        c.checkpoint_dir = k["checkpoint_dir"].as<std::string>("./checkpoints");
        c.save_interval = k["save_interval"].as<int>(5);
    }
    if (auto& l = y["logging"]) c.log_dir = l["log_dir"].as<std::string>("./logs");
    if (auto& e = y["experiment"]) {
        c.experiment_name = e["name"].as<std::string>(experiment);
        c.seed = e["seed"].as<int>(42);
    }
    if (y["experiments"] && y["experiments"][experiment]) {   // :150-160
        auto& ex = y["experiments"][experiment];
        if (ex["training"] && ex["training"]["batch_size"]) c.batch_size = ex["training"]["batch_size"].as<int>();
        if (ex["experiment"] && ex["experiment"]["name"]) c.experiment_name = ex["experiment"]["name"].as<std::string>();
    }
    if (auto& m = y["model"]) {   // :325-333 (architecture key ignored, like the reference)
        c.init_features = m["init_features"].as<int>(64);
        c.max_depth = m["max_depth"].as<float>(10.0f);
    }
    if (auto& d = y["data"]) {
        c.height = d["input_height"].as<int>(240);
        c.width = d["input_width"].as<int>(320);
        c.dataset = d["dataset_name"].as<std::string>("sunrgbd");
        c.n_train = d["num_train_samples"].as<int>(64);
        c.n_val = d["num_val_samples"].as<int>(16);
        c.manifest_path = d["manifest_path"].as<std::string>("./data/sunrgbd_manifest.json");
        if (auto& a = d["augmentation"]) {
            c.aug_crop = a["random_crop"].as<bool>(true);
            c.aug_flip = a["horizontal_flip"].as<bool>(true);
            c.aug_flip_p = a["flip_probability"].as<float>(0.5f);
            c.aug_jitter = a["color_jitter"].as<bool>(true);
            c.aug_brightness = a["brightness"].as<float>(0.2f);
            c.aug_contrast = a["contrast"].as<float>(0.2f);
        }
    }
    if (auto& hw = y["hardware"]) {
        c.distributed = hw["distributed"].as<bool>(false);
        c.num_gpus = hw["num_gpus"].as<int>(1);
        c.backend = hw["backend"].as<std::string>("nccl");
        for (float v : hw["gpu_ids"].as<std::vector<float>>({})) c.gpu_ids.push_back((int)v);
    }
    c.checkpoint_dir += "/" + c.experiment_name;   // :163-164
    c.log_dir += "/" + c.experiment_name;
    return c;
}

// ---- synthetic SUN-RGB-D-shaped samples (same generator as synthetic.py / SURVEY §8d) ----
uint64_t splitmix64(uint64_t seed, uint64_t idx) {
    uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
float u01(uint64_t seed, uint64_t idx) { return (float)((uint32_t)(splitmix64(seed, idx) >> 32) >> 8) * (1.0f / 16777216.0f); }

struct HostBatch {
    std::vector<float> rgb, gt, K;
};
// sample s of a split = sample s of one virtual batch (split offsets keep train/val disjoint)
void make_sample(int64_t s, int H, int W, float* rgb, float* gt, float* K) {
    const int64_t HW = (int64_t)H * W;
    for (int64_t i = 0; i < 3 * HW; ++i) rgb[i] = u01(0xC0FFEE, s * 3 * HW + i);
    for (int v = 0; v < H; ++v)
        for (int u = 0; u < W; ++u) {
            const int64_t idx = s * HW + (int64_t)v * W + u;
            double d = 0.5 + 9.0 * (0.5 + 0.5 * std::sin(2.0 * M_PI * ((double)u / W * 1.3 + (double)v / H * 0.7 + 0.1 * s)));
            d = std::min(9.5, std::max(0.5, d));
            if (u01(0xD3E7, idx) < 0.15f || v < H / 16) d = 0.0;
            gt[(int64_t)v * W + u] = (float)d;
        }
    const bool even = s % 2 == 0;
    const float sx = (float)W / 640.f, sy = (float)H / 480.f;
    std::fill(K, K + 9, 0.f);
    K[0] = (even ? 518.858f : 570.342f) * sx;
    K[2] = (even ? 325.582f : 320.0f) * sx;
    K[4] = (even ? 519.470f : 570.342f) * sy;
    K[5] = (even ? 253.736f : 240.0f) * sy;
    K[8] = 1.f;
}

bool ends_with(const std::string& s, const std::string& suf) {
    return s.size() >= suf.size() && s.compare(s.size() - suf.size(), suf.size(), suf) == 0;
}

// ---- checkpoint (.cadckpt): named tensors in reference layout + Adam state ----
void save_checkpoint(const std::string& path, BaselineUNetImpl& m, optim::Adam& opt) {
    std::ofstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot write checkpoint " + path);
    auto ps = m.named_parameters();
    auto bs = m.named_buffers();
    ps.insert(ps.end(), bs.begin(), bs.end());
    f.write("CADCKPT1", 8);
    int32_t n = (int32_t)ps.size();
    f.write((const char*)&n, 4);
    for (auto& t : ps) {
        int32_t ln = (int32_t)t.name.size(), nd = (int32_t)t.shape.size();
        f.write((const char*)&ln, 4);
        f.write(t.name.data(), ln);
        f.write((const char*)&nd, 4);
        f.write((const char*)t.shape.data(), 8 * nd);
        f.write((const char*)t.value.data(), 4 * (int64_t)t.value.size());
    }
    float *mp, *vp, *pp;
    int64_t nflat;
    cad::check(cad_unet_flat(m.handle(), &pp, nullptr, &nflat), "flat");
    cad::check(cad_adam_state(opt.handle(), &mp, &vp), "adam_state");
    std::vector<float> buf((size_t)nflat);
    int64_t step = opt.step_count();
    f.write("ADAM", 4);
    f.write((const char*)&step, 8);
    f.write((const char*)&nflat, 8);
    for (float* src : {mp, vp}) {
        cad::check(cad_memcpy(buf.data(), src, 4 * nflat, 1, nullptr), "d2h");
        f.write((const char*)buf.data(), 4 * nflat);
    }
}

void load_checkpoint(const std::string& path, BaselineUNetImpl& m, optim::Adam& opt) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("Cannot open checkpoint: " + path);
    char magic[8];
    f.read(magic, 8);
    if (std::memcmp(magic, "CADCKPT1", 8) != 0) throw std::runtime_error("not a .cadckpt file: " + path);
    int32_t n;
    f.read((char*)&n, 4);
    std::vector<NamedTensor> ts((size_t)n);
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
    if (m.load(ts) != n) throw std::runtime_error("checkpoint does not match the model: " + path);
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

// ---- data-parallel job: one process per GPU (hardware.distributed / num_gpus / gpu_ids,
// configs/train_config.yaml:176-183 — keys the reference parses but never uses) ----
constexpr const char* kEnvRank = "CAD_DP_RANK";
constexpr const char* kEnvWorld = "CAD_DP_WORLD";
constexpr const char* kEnvDevice = "CAD_DP_DEVICE";
constexpr const char* kEnvIdFile = "CAD_DP_ID_FILE";

struct Rank {
    int rank = 0, world = 1, device = 0;
    bool dp = false;        // a communicator is built (distributed: true, even for one GPU)
    std::string id_file;    // the launcher's rendezvous file ("" for a single process)
};

std::vector<int> dp_devices(const Config& c) {
    std::vector<int> ids = c.gpu_ids;
    if ((int)ids.size() < c.num_gpus) {
        ids.clear();
        for (int i = 0; i < c.num_gpus; ++i) ids.push_back(i);
    }
    ids.resize((size_t)c.num_gpus);
    return ids;
}

// The launcher: starts one child per GPU (this process makes no GPU call at all, so starting a fresh
// program is safe), forwards the exit status of the first child that fails, and stops the others
// then (a rank blocked in a collective would otherwise wait forever).
int launch_ranks(const Args& args, const Config& c) {
    const std::vector<int> devs = dp_devices(c);
    char tmpl[] = "/tmp/cad_dp_XXXXXX";
    if (!mkdtemp(tmpl)) throw std::runtime_error("cannot create the rendezvous directory");
    const std::string dir = tmpl, id_file = dir + "/rccl_id";
    std::vector<char*> argv;
    for (const auto& s : args.argv) argv.push_back(const_cast<char*>(s.c_str()));
    argv.push_back(nullptr);
    std::vector<pid_t> pids;
    for (int r = 0; r < c.num_gpus; ++r) {
        std::vector<std::string> env;
        for (char** e = environ; *e; ++e)
            if (std::strncmp(*e, "CAD_DP_", 7) != 0) env.push_back(*e);
        env.push_back(std::string(kEnvRank) + "=" + std::to_string(r));
        env.push_back(std::string(kEnvWorld) + "=" + std::to_string(c.num_gpus));
        env.push_back(std::string(kEnvDevice) + "=" + std::to_string(devs[(size_t)r]));
        env.push_back(std::string(kEnvIdFile) + "=" + id_file);
        std::vector<char*> envp;
        for (auto& e : env) envp.push_back(const_cast<char*>(e.c_str()));
        envp.push_back(nullptr);
        pid_t pid;
        if (posix_spawn(&pid, "/proc/self/exe", nullptr, nullptr, argv.data(), envp.data()) != 0) {
            for (pid_t p : pids) kill(p, SIGTERM);
            throw std::runtime_error("cannot start rank " + std::to_string(r));
        }
        pids.push_back(pid);
    }
    int rc = 0;
    for (size_t left = pids.size(); left > 0; --left) {
        int st = 0;
        const pid_t p = waitpid(-1, &st, 0);
        if (p < 0) break;
        const int code = WIFEXITED(st) ? WEXITSTATUS(st) : 128 + (WIFSIGNALED(st) ? WTERMSIG(st) : 0);
        if (code != 0 && rc == 0) {
            rc = code;
            std::cerr << "rank " << (std::find(pids.begin(), pids.end(), p) - pids.begin()) << " failed (status "
                      << code << "); stopping the other ranks\n";
            for (pid_t q : pids)
                if (q != p) kill(q, SIGTERM);
        }
    }
    std::error_code ec;
    fs::remove_all(dir, ec);
    return rc;
}

Rank rank_of_process(const Config& c, const Args& args) {
    Rank r;
    if (const char* e = std::getenv(kEnvRank)) {
        r.rank = std::atoi(e);
        r.world = std::atoi(std::getenv(kEnvWorld) ? std::getenv(kEnvWorld) : "1");
        r.device = std::atoi(std::getenv(kEnvDevice) ? std::getenv(kEnvDevice) : "0");
        r.id_file = std::getenv(kEnvIdFile) ? std::getenv(kEnvIdFile) : "";
        r.dp = true;
        if (r.world < 1 || r.rank < 0 || r.rank >= r.world || r.id_file.empty())
            throw std::runtime_error("inconsistent data-parallel rank environment");
    } else {
        r.device = c.distributed && !c.gpu_ids.empty() ? c.gpu_ids[0] : args.gpu;
        r.dp = c.distributed;   // one GPU, distributed: a single-rank communicator
    }
    return r;
}

// RCCL id rendezvous through the launcher's file: rank 0 writes it (write, then rename: readers never
// see a partial file), the others poll for it.  A dry run exchanges random bytes instead.
distributed::UniqueId exchange_id(const Rank& r, bool dry) {
    distributed::UniqueId id{};
    auto draw = [&] {
        if (!dry) return distributed::Communicator::unique_id();
        std::random_device rd;
        distributed::UniqueId x{};
        for (auto& b : x) b = (uint8_t)rd();
        return x;
    };
    if (r.id_file.empty()) return draw();
    if (r.rank == 0) {
        id = draw();
        const std::string tmp = r.id_file + ".tmp";
        {
            std::ofstream f(tmp, std::ios::binary);
            f.write(reinterpret_cast<const char*>(id.data()), (std::streamsize)id.size());
            if (!f) throw std::runtime_error("cannot write " + tmp);
        }
        fs::rename(tmp, r.id_file);
        return id;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        std::error_code ec;
        if (fs::exists(r.id_file, ec) && fs::file_size(r.id_file, ec) == id.size()) {
            std::ifstream f(r.id_file, std::ios::binary);
            f.read(reinterpret_cast<char*>(id.data()), (std::streamsize)id.size());
            if (f) return id;
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(300))
            throw std::runtime_error("rank " + std::to_string(r.rank) + ": no communicator id from rank 0");
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
}

// global batch bi = samples [bi*B*world, (bi+1)*B*world); rank r takes its r-th B-slice.  With more
// than one rank the last partial global batch is dropped (every replica must step together).
struct Shard {
    int64_t first;
    int n;
};
int steps_per_epoch(int n_train, int B, int world) {
    return world > 1 ? n_train / (B * world) : (n_train + B - 1) / B;
}
Shard shard_of(int bi, int n_train, int B, const Rank& r) {
    const int64_t first = (int64_t)bi * B * r.world + (int64_t)r.rank * B;
    return {first, (int)std::min<int64_t>(B, n_train - first)};
}

int dry_run(const Config& c, const Rank& r) {
    const auto id = exchange_id(r, true);
    uint64_t h = 1469598103934665603ull;   // FNV-1a of the rendezvous bytes: equal on every rank
    for (uint8_t b : id) h = (h ^ b) * 1099511628211ull;
    int ns = 0;
    int64_t off[16], cnt[16], n_flat = 0;
    cad::check(cad_model_grad_layout(CAD_MODEL_BASELINE, 3, c.init_features, &ns, off, cnt, &n_flat), "layout");
    int64_t boff[16], bcnt[16];
    int blast[16];
    const int nb = cad_plan_grad_buckets(off, cnt, ns, 25 << 18, boff, bcnt, blast);
    const int spe = steps_per_epoch(c.n_train, c.batch_size, r.world);
    std::ostringstream o;
    o << "{\"rank\": " << r.rank << ", \"world\": " << r.world << ", \"device\": " << r.device
      << ", \"communicator\": " << (r.dp ? "true" : "false") << ", \"id_hash\": " << h
      << ", \"steps_per_epoch\": " << spe << ", \"global_batch\": " << c.batch_size * r.world << ", \"first_step_samples\": [";
    const Shard s0 = shard_of(0, c.n_train, c.batch_size, r);
    o << s0.first << ", " << s0.first + s0.n << "], \"n_flat\": " << n_flat << ", \"buckets\": [";
    for (int i = 0; i < nb; ++i) o << (i ? ", " : "") << "[" << boff[i] << ", " << bcnt[i] << ", " << blast[i] << "]";
    o << "]}";
    std::cout << o.str() << std::endl;
    return 0;
}

int run(const Args& args) {
    yaml_lite::Node y = yaml_lite::load_file(args.config);
    Config c = load_config(y, args.experiment);
    if (args.debug || (y["debug"] && y["debug"]["enabled"].as<bool>(false))) {   // :297-301
        c.num_epochs = y["debug"]["num_epochs"].as<int>(2);
        c.log_interval = y["debug"]["log_interval"].as<int>(1);
    }
    if (c.distributed && c.backend != "nccl" && c.backend != "rccl")
        throw std::runtime_error("hardware.backend '" + c.backend + "': this build exchanges gradients over RCCL (\"nccl\")");
    if (c.distributed && c.num_gpus > 1 && !std::getenv(kEnvRank)) return launch_ranks(args, c);
    const Rank R = rank_of_process(c, args);
    // the dataset: "synthetic" = generated batches; anything else = the SUN RGB-D manifest through the
    // prefetch ring (cad_dataset / cad_loader: decode on host threads, pinned double-buffered upload,
    // resize + augmentation on device).  Like the reference, train and validation read the same
    // manifest (its split argument is unused, sunrgbd_loader.cpp:39-78); validation takes the first
    // min(500, size) samples (validateEpoch :343) without augmentation.
    const bool real = c.dataset != "synthetic";
    std::unique_ptr<cad_dataset, void (*)(cad_dataset*)> ds(nullptr, cad_dataset_destroy);
    if (real) {
        cad_dataset* d = nullptr;
        cad::check(cad_dataset_open(c.manifest_path.c_str(), nullptr, 0, &d), "SunRGBDLoader");
        ds.reset(d);
        c.n_train = (int)cad_dataset_size(d);
        c.n_val = std::min(500, c.n_train);
        if (c.n_train == 0) throw std::runtime_error("no usable samples in " + c.manifest_path);
    }
    if (args.dry_run) return dry_run(c, R);
    const bool lead = R.rank == 0;   // logs, validation and checkpoints (rank 0's replica)
    if (lead) std::cout << "Loading configuration from: " << args.config << "\n";
    if (args.debug && lead) std::cout << "Debug mode enabled - using reduced dataset\n";
    int ndev = 0;
    cad::check(cad_device_count(&ndev), "device query");
    if (R.device < 0 || R.device >= ndev) throw std::runtime_error("GPU " + std::to_string(R.device) + " not available");
    cad::check(cad_set_device(R.device), "set device");
    if (lead) {
        fs::create_directories(c.checkpoint_dir);
        fs::create_directories(c.log_dir);
    }

    const int B = c.batch_size, H = c.height, W = c.width;
    cad::Workspace ws{B, H, W, R.device};
    BaselineUNetImpl model(3, c.init_features, c.max_depth, ws);
    CombinedDepthLoss loss_fn(c.si, c.grad, c.smooth, c.reproj, ws);
    optim::Adam opt(model, c.learning_rate, c.weight_decay);
    std::unique_ptr<distributed::Communicator> comm;
    if (R.dp) comm = std::make_unique<distributed::Communicator>(exchange_id(R, false), R.world, R.rank, R.device);
    if (lead)
        std::cout << "Model: baseline_unet (f=" << c.init_features << "), parameters: " << model.count_parameters() << "\n"
                  << "Using MI355X device " << R.device
                  << (R.dp ? " (data-parallel rank 0 of " + std::to_string(R.world) + ", RCCL)" : std::string()) << "\n"
                  << "Training samples: " << c.n_train << (real ? " (" + c.manifest_path + ")" : std::string(" (synthetic)"))
                  << ", validation samples: " << c.n_val << "\n";
    if (!args.resume.empty()) {
        if (ends_with(args.resume, ".pt")) {   // a torch::save model archive (ours or the reference's)
            load(model, args.resume);
            if (lead) std::cout << "Loaded model weights from " << args.resume << " (optimizer state starts fresh)\n";
        } else {
            load_checkpoint(args.resume, model, opt);
            if (lead) std::cout << "Resumed from " << args.resume << " (optimizer step " << opt.step_count() << ")\n";
        }
    }
    if (comm) comm->broadcast_parameters(model, 0);   // identical replicas

    std::ofstream train_log, metrics_csv, tb;
    if (lead) {
        train_log.open(c.log_dir + "/training.log", std::ios::app);
        metrics_csv.open(c.log_dir + "/metrics.csv", std::ios::app);
        if (metrics_csv.tellp() == 0)
            metrics_csv << "epoch,step,train_loss,val_loss,abs_rel,sq_rel,rmse,rmse_log,a1,a2,a3,learning_rate,time_elapsed\n";
        if (args.tensorboard) {
            tb.open(c.log_dir + "/tensorboard_scalars.csv", std::ios::app);
            if (tb.tellp() == 0) tb << "tag,step,value\n";
        }
    }

    const int64_t HW = (int64_t)H * W;
    HostBatch hb;
    hb.rgb.resize((size_t)(B * 3 * HW));
    hb.gt.resize((size_t)(B * HW));
    hb.K.resize((size_t)B * 9);
    DeviceTensor rgb = DeviceTensor::empty({B, 3, H, W}, R.device), gt = DeviceTensor::empty({B, 1, H, W}, R.device),
                 K = DeviceTensor::empty({B, 3, 3}, R.device), pred = DeviceTensor::empty({B, 1, H, W}, R.device);
    auto upload = [&](int64_t first, int n, int64_t split_offset) {
        for (int i = 0; i < n; ++i)
            make_sample(split_offset + first + i, H, W, hb.rgb.data() + i * 3 * HW, hb.gt.data() + i * HW, hb.K.data() + i * 9);
        cad::check(cad_memcpy(rgb.data, hb.rgb.data(), 4 * n * 3 * HW, 0, nullptr), "h2d");
        cad::check(cad_memcpy(gt.data, hb.gt.data(), 4 * n * HW, 0, nullptr), "h2d");
        cad::check(cad_memcpy(K.data, hb.K.data(), 4 * n * 9, 0, nullptr), "h2d");
        rgb.shape[0] = gt.shape[0] = K.shape[0] = pred.shape[0] = n;
    };
    std::unique_ptr<cad_loader, void (*)(cad_loader*)> train_L(nullptr, cad_loader_destroy), val_L(nullptr, cad_loader_destroy);
    if (real) {
        cad_aug_config ac{};
        ac.enable_random_crop = c.aug_crop; ac.crop_scale_min = 0.7f; ac.crop_scale_max = 1.0f;
        ac.enable_horizontal_flip = c.aug_flip; ac.horizontal_flip_prob = c.aug_flip_p;
        ac.enable_color_jitter = c.aug_jitter; ac.brightness_delta = c.aug_brightness; ac.contrast_delta = c.aug_contrast;
        const int threads = (int)std::max(2u, std::min(8u, std::thread::hardware_concurrency()));
        cad_loader* L = nullptr;
        cad::check(cad_loader_create(ds.get(), B, H, W, &ac, 42, threads, 2, R.device, &L), "train loader");
        train_L.reset(L);
        cad::check(cad_loader_create(ds.get(), B, H, W, nullptr, 42, threads, 2, R.device, &L), "val loader");
        val_L.reset(L);
    }
    auto fetch = [&](cad_loader* L, int expect) {
        const int n = cad_loader_next(L, rgb.data, gt.data, K.data, nullptr);
        if (n < 0) throw std::runtime_error(std::string("data loader: ") + cad_last_error());
        if (n != expect) throw std::runtime_error("data loader: batch of " + std::to_string(n) + ", expected " + std::to_string(expect));
        rgb.shape[0] = gt.shape[0] = K.shape[0] = pred.shape[0] = n;
    };
    const auto t0 = std::chrono::steady_clock::now();
    int64_t global_step = opt.step_count();
    const int nb = steps_per_epoch(c.n_train, B, R.world);
    if (nb < 1) throw std::runtime_error("fewer training samples than one global batch");
    const int start_epoch = 1 + (int)(global_step / nb);
    constexpr int64_t kBucketElems = 25 << 18;   // 25 MB gradient buckets
    for (int epoch = start_epoch; epoch <= c.num_epochs; ++epoch) {
        model.train();
        double total = 0.0;
        int64_t seen = 0;
        if (real) {   // this rank's samples of the epoch, in step order
            std::vector<int64_t> order;
            for (int bi = 0; bi < nb; ++bi) {
                const Shard sh = shard_of(bi, c.n_train, B, R);
                for (int j = 0; j < sh.n; ++j) order.push_back(sh.first + j);
            }
            cad::check(cad_loader_start_epoch(train_L.get(), order.data(), (int64_t)order.size()), "start epoch");
        }
        for (int bi = 0; bi < nb; ++bi) {   // enhanced.h:266-329
            const Shard sh = shard_of(bi, c.n_train, B, R);   // last partial batch (:269-270) on one rank
            if (real) fetch(train_L.get(), sh.n);
            else upload(sh.first, sh.n, 0);
            opt.zero_grad();
            model.forward_into(rgb, pred);
            DeviceTensor l = loss_fn.forwardWithIntrinsics(pred, gt, rgb, K);
            if (comm) comm->backward_allreduce(model, loss_fn.dpred(), kBucketElems);
            else model.backward(loss_fn.dpred());
            // clip_grad_norm_ on the mean gradient (the SUM all-reduce's 1/world folded in)
            const double gnorm = c.use_grad_clip ? clip_grad_norm_(model, c.grad_clip_value, nullptr, 1.0 / R.world) : 0.0;
            if (!c.use_grad_clip)
                cad::check(cad_clip_grad_norm(model.handle(), INFINITY, 1.f / R.world, nullptr), "noclip");
            opt.step();
            if (comm) comm->allreduce(l.data, 5);   // the logged loss: mean over replicas
            const float lv = l.to_host()[0] / R.world;   // loss.item<float>() (:307)
            if (!std::isfinite(lv)) throw std::runtime_error("non-finite loss at step " + std::to_string(global_step));
            total += (double)lv * sh.n * R.world;
            seen += (int64_t)sh.n * R.world;
            ++global_step;
            if (lead && ((bi + 1) % c.log_interval == 0 || bi == nb - 1)) {
                std::cout << "\r  [" << (100 * (bi + 1) / nb) << "%] Batch " << (bi + 1) << "/" << nb
                          << " | Loss: " << lv << std::flush;
                if (tb) tb << "batch_loss/train," << global_step << "," << lv << "\ntraining/gradient_norm,"
                           << global_step << "," << gnorm << "\n";
            }
        }
        if (!lead) continue;   // validation, logs and checkpoints: rank 0 (identical replicas)
        std::cout << "\n";
        const float train_loss = (float)(total / std::max<int64_t>(1, seen));
        float val_loss = 0.f;
        DepthMetrics vm{};
        if (c.val_interval > 0 && epoch % c.val_interval == 0 && c.n_val > 0) {   // validateEpoch :339-395
            model.eval();
            double vl = 0.0;
            int vn = 0;
            if (real) cad::check(cad_loader_start_epoch(val_L.get(), nullptr, c.n_val), "validation");
            for (int64_t s = 0; s < c.n_val; s += B) {
                const int n = (int)std::min<int64_t>(B, c.n_val - s);
                if (real) fetch(val_L.get(), n);
                else upload(s, n, 1 << 20);
                model.forward_into(rgb, pred);
                DeviceTensor l = loss_fn.forwardWithIntrinsics(pred, gt, rgb, K);
                // the reference evaluates sample by sample (batch 1); loss over a batch of n equals the
                // per-sample mean only for n == 1, so report the batch loss weighted by n
                vl += (double)l.to_host()[0] * n;
                DepthMetrics m = computeDepthMetrics(pred, gt);
                vm.abs_rel += m.abs_rel * n; vm.sq_rel += m.sq_rel * n; vm.rmse += m.rmse * n;
                vm.rmse_log += m.rmse_log * n; vm.a1 += m.a1 * n; vm.a2 += m.a2 * n; vm.a3 += m.a3 * n;
                vn += n;
            }
            val_loss = (float)(vl / vn);
            for (float* p : {&vm.abs_rel, &vm.sq_rel, &vm.rmse, &vm.rmse_log, &vm.a1, &vm.a2, &vm.a3}) *p /= vn;
        }
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        metrics_csv << epoch << "," << global_step << "," << train_loss << "," << val_loss << "," << vm.abs_rel << ","
                    << vm.sq_rel << "," << vm.rmse << "," << vm.rmse_log << "," << vm.a1 << "," << vm.a2 << "," << vm.a3
                    << "," << c.learning_rate << "," << el << "\n";
        metrics_csv.flush();
        train_log << "Epoch " << epoch << " train_loss " << train_loss << " val_loss " << val_loss << " abs_rel "
                  << vm.abs_rel << "\n";
        if (tb) tb << "loss/train," << epoch << "," << train_loss << "\nloss/val," << epoch << "," << val_loss
                   << "\nmetrics/abs_rel," << epoch << "," << vm.abs_rel << "\n";
        std::cout << "Epoch " << epoch << "/" << c.num_epochs << " | train " << train_loss << " | val " << val_loss
                  << " | abs_rel " << vm.abs_rel << " | " << el << " s\n";
        if (c.save_interval > 0 && epoch % c.save_interval == 0) {
            // the reference's checkpoint, torch::save(model_, <dir>/<exp>_epoch_N.pt) (enhanced.h:656-662),
            // plus the optimizer state it never saves (.cadckpt: full resume)
            const std::string stem = c.checkpoint_dir + "/" + c.experiment_name + "_epoch_" + std::to_string(epoch);
            save(model, stem + ".pt");
            save_checkpoint(stem + ".cadckpt", model, opt);
            std::cout << "Checkpoint saved: " << stem << ".pt\n";
        }
    }
    if (lead) {
        save(model, c.checkpoint_dir + "/final_model.pt");   // production_trainer.h:323-330
        save_checkpoint(c.checkpoint_dir + "/final_model.cadckpt", model, opt);
        std::cout << "Training complete.\n";
    }
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    try {
        return run(parse_args(argc, argv));
    } catch (const std::exception& e) {
        std::cerr << "Error: " << e.what() << std::endl;   // train_main.cpp:503-506
        return 1;
    }
}

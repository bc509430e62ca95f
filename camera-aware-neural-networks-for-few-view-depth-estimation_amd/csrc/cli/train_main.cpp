// build/train — drop-in for the reference's `./build/train --config <yaml>` entry point
// (src/training/train_main.cpp:279-507 driving TensorBoardTrainerEnhanced, enhanced.h:142-334),
// on libcad_hip.so through the C++ drop-in classes of include/cad/cad.hpp and the trainer of
// include/cad/trainer.hpp (SunRGBDLoader + TensorBoardTrainerEnhanced).
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
// model.architecture selects the FiLM models and the geometry-aware networks (model.variant,
// use_pcl, use_attention; single process) — the reference always builds BaselineUNet;
// data.dataset_name "synthetic" trains on generated samples, anything else on the manifest's PNG / PNM /
// JPEG files (csrc/host/jpeg.cpp decodes as cv::imread does); hardware.distributed runs DP over RCCL.
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
#include "../../../include/cad/trainer.hpp"
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
    std::string dataset = "sunrgbd", data_dir = "./data/sunrgbd";
    std::string manifest_path = "./data/sunrgbd_manifest.json";
    std::vector<std::string> sensor_types;   // data.sensor_types (empty: all four)
    std::string architecture = "baseline_unet";
    std::string variant = "full";             // model.variant (geometry_aware: "full" / "lightweight")
    bool use_pcl = true, use_attention = true;
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
    if (auto& m = y["model"]) {   // :325-333
        c.init_features = m["init_features"].as<int>(64);
        c.max_depth = m["max_depth"].as<float>(10.0f);
        // the reference parses model.architecture and always builds BaselineUNet; here it selects the
        // FiLM models of configs 3 (intrinsics_unet: FiLM blocks; ray_film_unet: + ray-enhanced enc1)
        c.architecture = m["architecture"].as<std::string>("baseline_unet");
        if (c.architecture != "baseline_unet" && c.architecture != "intrinsics_unet" && c.architecture != "ray_film_unet" &&
            c.architecture != "geometry_aware")
            throw std::runtime_error("model.architecture '" + c.architecture +
                                     "': this CLI trains baseline_unet, intrinsics_unet, ray_film_unet or geometry_aware");
        // geometry_aware (train_config.yaml:51-57 and its experiments): model.variant full /
        // lightweight, use_pcl, use_attention (GeometryAwareNetworkImpl / LightweightGeometryNetworkImpl)
        c.variant = m["variant"].as<std::string>("full");
        c.use_pcl = m["use_pcl"].as<bool>(true);
        c.use_attention = m["use_attention"].as<bool>(true);
        if (c.architecture == "geometry_aware" && c.variant != "full" && c.variant != "lightweight")
            throw std::runtime_error("model.variant '" + c.variant + "': expected full or lightweight");
    }
    if (auto& d = y["data"]) {
        c.height = d["input_height"].as<int>(240);
        c.width = d["input_width"].as<int>(320);
        c.dataset = d["dataset_name"].as<std::string>("sunrgbd");
        c.n_train = d["num_train_samples"].as<int>(64);
        c.n_val = d["num_val_samples"].as<int>(16);
        c.manifest_path = d["manifest_path"].as<std::string>("./data/sunrgbd_manifest.json");
        c.data_dir = d["data_dir"].as<std::string>("./data/sunrgbd");
        c.sensor_types = d["sensor_types"].as<std::vector<std::string>>({});
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

bool ends_with(const std::string& s, const std::string& suf) {
    return s.size() >= suf.size() && s.compare(s.size() - suf.size(), suf.size(), suf) == 0;
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
    if (real) {   // the sample count, read on the host before any GPU call
        std::vector<const char*> sens;
        for (const auto& x : c.sensor_types) sens.push_back(x.c_str());
        cad_dataset* d = nullptr;
        cad::check(cad_dataset_open(c.manifest_path.c_str(), sens.empty() ? nullptr : sens.data(), (int)sens.size(), &d),
                   "SunRGBDLoader");
        c.n_train = (int)cad_dataset_size(d);
        cad_dataset_destroy(d);
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

    // the loaders (train_main.cpp:366-395): both splits read the same manifest (the reference's split
    // argument is unused); train augments (AugmentationConfig from data.augmentation, seed 42)
    std::shared_ptr<SunRGBDLoader> train_loader, val_loader;
    if (real) {
        train_loader = std::make_shared<SunRGBDLoader>(c.data_dir, c.manifest_path, "train");
        val_loader = std::make_shared<SunRGBDLoader>(c.data_dir, c.manifest_path, "test");
        if (!c.sensor_types.empty()) {
            train_loader->filterBySensorType(c.sensor_types);
            val_loader->filterBySensorType(c.sensor_types);
        }
        AugmentationConfig ac;
        ac.enable_random_crop = c.aug_crop;
        ac.enable_horizontal_flip = c.aug_flip;
        ac.horizontal_flip_prob = c.aug_flip_p;
        ac.enable_color_jitter = c.aug_jitter;
        ac.brightness_delta = c.aug_brightness;
        ac.contrast_delta = c.aug_contrast;
        train_loader->enableAugmentation(ac);
    } else {   // disjoint generated splits
        train_loader = SunRGBDLoader::synthetic(c.n_train, c.height, c.width, (uint32_t)c.seed);
        if (c.n_val > 0) val_loader = SunRGBDLoader::synthetic(c.n_val, c.height, c.width, (uint32_t)c.seed + 1);
    }
    for (auto& L : {train_loader, val_loader})
        if (L) L->setTargetDimensions(c.height, c.width);

    cad::Workspace ws{c.batch_size, c.height, c.width, R.device};
    if (c.architecture == "geometry_aware") {   // single-process GeometryTrainer (trainer.hpp)
        if (R.dp) throw std::runtime_error("geometry_aware trains on one GPU here (hardware.distributed: false)");
        if (!args.resume.empty()) throw std::runtime_error("--resume is not supported for geometry_aware");
        std::shared_ptr<GeometryAwareNetworkImpl> geo;
        if (c.variant == "lightweight")
            geo = std::make_shared<LightweightGeometryNetworkImpl>(3, c.init_features, 4, c.max_depth, ws);
        else
            geo = std::make_shared<GeometryAwareNetworkImpl>(3, c.init_features, 4, c.max_depth, c.use_pcl,
                                                             c.use_attention, ws);
        auto gloss = std::make_shared<CombinedDepthLoss>(c.si, c.grad, c.smooth, c.reproj, ws);
        std::cout << "Model: geometry_aware/" << c.variant << " (f=" << c.init_features << ", pcl " << c.use_pcl
                  << ", attention " << c.use_attention << "), parameters: " << geo->count_parameters()
                  << "\nUsing MI355X device " << R.device << "\nTraining samples: " << c.n_train
                  << (real ? " (" + c.manifest_path + ")" : std::string(" (synthetic)")) << "\n";
        TensorBoardTrainerEnhanced::Config gc;
        gc.num_epochs = c.num_epochs;
        gc.batch_size = c.batch_size;
        gc.learning_rate = c.learning_rate;
        gc.weight_decay = c.weight_decay;
        gc.use_grad_clip = c.use_grad_clip;
        gc.grad_clip_value = c.grad_clip_value;
        gc.val_interval = c.val_interval;
        gc.log_interval = c.log_interval;
        gc.save_interval = c.save_interval;
        gc.checkpoint_dir = c.checkpoint_dir;
        gc.log_dir = c.log_dir;
        gc.experiment_name = c.experiment_name;
        gc.device = R.device;
        GeometryTrainer gt(geo, gloss, gc);
        gt.train(train_loader, val_loader);
        std::cout << "Training complete.\n";
        return 0;
    }
    std::shared_ptr<BaselineUNetImpl> model;
    if (c.architecture == "intrinsics_unet")
        model = std::make_shared<IntrinsicsConditionedUNetImpl>(3, c.init_features, 4, c.max_depth, ws);
    else if (c.architecture == "ray_film_unet")
        model = std::make_shared<RayConditionedUNetImpl>(3, c.init_features, 4, c.max_depth, ws);
    else
        model = std::make_shared<BaselineUNetImpl>(3, c.init_features, c.max_depth, ws);
    auto loss_fn = std::make_shared<CombinedDepthLoss>(c.si, c.grad, c.smooth, c.reproj, ws);
    std::shared_ptr<distributed::Communicator> comm;
    if (R.dp) comm = std::make_shared<distributed::Communicator>(exchange_id(R, false), R.world, R.rank, R.device);
    if (lead)
        std::cout << "Model: " << c.architecture << " (f=" << c.init_features << "), parameters: " << model->count_parameters()
                  << "\nUsing MI355X device " << R.device
                  << (R.dp ? " (data-parallel rank 0 of " + std::to_string(R.world) + ", RCCL)" : std::string()) << "\n"
                  << "Training samples: " << c.n_train << (real ? " (" + c.manifest_path + ")" : std::string(" (synthetic)"))
                  << ", validation samples: " << (real ? std::min(500, c.n_train) : c.n_val) << "\n";

    TensorBoardTrainerEnhanced::Config tc;   // train_main.cpp:436-458
    tc.num_epochs = c.num_epochs;
    tc.batch_size = c.batch_size;
    tc.learning_rate = c.learning_rate;
    tc.weight_decay = c.weight_decay;
    tc.use_grad_clip = c.use_grad_clip;
    tc.grad_clip_value = c.grad_clip_value;
    tc.val_interval = c.val_interval;
    tc.log_interval = c.log_interval;
    tc.save_interval = c.save_interval;
    tc.checkpoint_dir = c.checkpoint_dir;
    tc.log_dir = c.log_dir;
    tc.experiment_name = c.experiment_name;
    tc.device = R.device;
    tc.tensorboard = args.tensorboard;
    TensorBoardTrainerEnhanced trainer(model, model, loss_fn, tc, comm);
    if (!args.resume.empty()) {
        trainer.loadCheckpoint(args.resume);
        if (lead) {
            if (ends_with(args.resume, ".pt"))   // a torch::save model archive (ours or the reference's)
                std::cout << "Loaded model weights from " << args.resume << " (optimizer state starts fresh)\n";
            else
                std::cout << "Resumed from " << args.resume << " (optimizer step " << trainer.optimizer().step_count() << ")\n";
        }
    }
    trainer.train(train_loader, val_loader);
    if (lead) std::cout << "Training complete.\n";
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

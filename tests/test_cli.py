"""Drop-in CLI (build/train, the reference's ./build/train --config) and its YAML-subset reader.
CPU: flags, error behaviour (train_main.cpp:503-506: "Error: <what>", exit 1), YAML parity with
PyYAML on the shipped configs.  GPU: a short synthetic run, metrics.csv, checkpoints, resume."""
import ctypes as C
import json
import os
import subprocess

import pytest
import yaml

from conftest import ROOT

PKG = os.path.join(ROOT, "camera-aware-neural-networks-for-few-view-depth-estimation_amd")
TRAIN = os.path.join(ROOT, "build", "train")


@pytest.fixture(scope="module")
def train_bin():
    # (-o libcad_hip.so: the library is never rebuilt here — on a GPU box its object files are absent,
    # and a rebuild would recompile every kernel inside the test session)
    subprocess.run(["make", "-C", PKG, "-o", "libcad_hip.so", "train"], check=True, capture_output=True)
    return TRAIN


def _flatten(d, path=""):
    out = {}
    if isinstance(d, dict):
        for k, v in d.items():
            out.update(_flatten(v, f"{path}.{k}" if path else str(k)))
    elif isinstance(d, list):
        for i, v in enumerate(d):
            out.update(_flatten(v, f"{path}[{i}]"))
    else:
        out[path] = d
    return out


@pytest.mark.parametrize("dumped", [False, True])
@pytest.mark.parametrize("cfg", ["train_config.yaml", "train_config_mi355x.yaml"])
def test_yaml_lite_matches_pyyaml(tmp_path, cfg, dumped):
    """The shipped configs as written, and re-emitted by yaml.safe_dump (block lists at the key's own
    indentation, quoting chosen by PyYAML) — the form tools that rewrite configs produce."""
    exe = tmp_path / "yaml_probe"
    subprocess.run(["g++", "-std=c++17", "-O1", "-o", str(exe), os.path.join(ROOT, "tests", "yaml_probe.cpp")],
                   check=True)
    path = os.path.join(ROOT, "configs", cfg)
    if dumped:
        d = yaml.safe_load(open(path))
        d.setdefault("hardware", {})["gpu_ids"] = [3, 5]
        d["hardware"]["nested"] = [{"a": 1, "b": [1, 2]}, {"c": "x y"}]
        path = tmp_path / cfg
        path.write_text(yaml.safe_dump(d))
    out = subprocess.run([str(exe), path], check=True, capture_output=True, text=True).stdout
    ours = dict(line.split("=", 1) for line in out.strip().splitlines())
    ref = _flatten(yaml.safe_load(open(path)))
    assert set(ours) == set(ref)
    for k, v in ref.items():
        if isinstance(v, bool):
            assert ours[k] in ("true", "false") and (ours[k] == "true") == v, k
        elif isinstance(v, (int, float)):
            assert abs(float(ours[k]) - v) <= 1e-12 * max(1.0, abs(v)), k
        else:
            assert ours[k] == str(v), k


def test_cli_help_and_errors(train_bin):
    r = subprocess.run([train_bin, "--help"], capture_output=True, text=True)
    assert r.returncode == 0 and "--config" in r.stdout
    r = subprocess.run([train_bin, "-c", "/nonexistent.yaml"], capture_output=True, text=True)
    assert r.returncode == 1 and r.stderr.startswith("Error: Cannot open config file")
    r = subprocess.run([train_bin, "--bogus"], capture_output=True, text=True)
    assert r.returncode == 1 and "Error:" in r.stderr


@pytest.mark.gpu
def test_cli_train_resume(train_bin, tmp_path):
    cfg = yaml.safe_load(open(os.path.join(ROOT, "configs", "train_config.yaml")))
    cfg["data"].update(num_train_samples=24, num_val_samples=8, input_height=64, input_width=96)
    cfg["training"].update(num_epochs=2, batch_size=8)
    cfg["checkpointing"]["checkpoint_dir"] = str(tmp_path / "ckpt")
    cfg["logging"]["log_dir"] = str(tmp_path / "logs")
    p = tmp_path / "cfg.yaml"
    p.write_text(yaml.safe_dump(cfg))
    r = subprocess.run([train_bin, "-c", str(p)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    rows = (tmp_path / "logs" / "baseline_unet" / "metrics.csv").read_text().strip().splitlines()
    assert rows[0].startswith("epoch,step,train_loss,val_loss,abs_rel")
    assert len(rows) == 3
    ck = tmp_path / "ckpt" / "baseline_unet"
    assert (ck / "baseline_unet_epoch_2.cadckpt").exists() and (ck / "final_model.cadckpt").exists()
    # the reference's checkpoint files, torch::save archives (enhanced.h:656-662): PyTorch reads them
    for name in ("baseline_unet_epoch_2.pt", "final_model.pt"):
        import torch
        sd = torch.jit.load(str(ck / name)).state_dict()
        assert len(sd) == 18 + 18 * 5 + 4 * 2 + 2 and int(sd["enc1.bn1.num_batches_tracked"]) == 6
    # weights-only start from a .pt (optimizer fresh)
    r = subprocess.run([train_bin, "-c", str(p), "-r", str(ck / "final_model.pt")], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and "Loaded model weights" in r.stdout, r.stderr
    # resume: continue to epoch 3 from the saved optimizer state
    cfg["training"]["num_epochs"] = 3
    p.write_text(yaml.safe_dump(cfg))
    r = subprocess.run([train_bin, "-c", str(p), "-r", str(ck / "final_model.cadckpt")], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "optimizer step 6" in r.stdout
    rows = (tmp_path / "logs" / "baseline_unet" / "metrics.csv").read_text().strip().splitlines()
    # the step column is the reference's global_step_ at logEpochMetrics: steps before this epoch
    # (enhanced.h:230-233)
    assert rows[-1].startswith("3,6,")


def _dp_cfg(tmp_path, **hw):
    cfg = {"data": {"dataset_name": "synthetic", "num_train_samples": 100, "num_val_samples": 8, "input_height": 64,
                    "input_width": 64},
           "model": {"init_features": 16}, "training": {"batch_size": 8, "num_epochs": 1},
           "hardware": dict({"device": "cuda", "gpu_ids": [3, 5], "num_gpus": 2, "distributed": True,
                             "backend": "nccl"}, **hw)}
    p = tmp_path / "dp.yaml"
    p.write_text(yaml.safe_dump(cfg))
    return p


def test_cli_model_architecture_key(train_bin, tmp_path):
    """model.architecture selects the network (the reference parses it and always builds BaselineUNet),
    model.variant the geometry-aware one; an architecture / variant this build does not train is
    refused before any GPU call."""
    p = _dp_cfg(tmp_path, distributed=False)
    cfg = yaml.safe_load(p.read_text())
    cfg["model"]["architecture"] = "vision_transformer"
    p.write_text(yaml.safe_dump(cfg))
    r = subprocess.run([train_bin, "-c", str(p), "--dry-run"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and r.stderr.startswith("Error: model.architecture 'vision_transformer'")
    cfg["model"].update(architecture="geometry_aware", variant="tiny")
    p.write_text(yaml.safe_dump(cfg))
    r = subprocess.run([train_bin, "-c", str(p), "--dry-run"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and r.stderr.startswith("Error: model.variant 'tiny'")
    cfg["model"]["variant"] = "lightweight"
    for arch in ("baseline_unet", "intrinsics_unet", "ray_film_unet", "geometry_aware"):
        cfg["model"]["architecture"] = arch
        p.write_text(yaml.safe_dump(cfg))
        r = subprocess.run([train_bin, "-c", str(p), "--dry-run"], capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, (arch, r.stderr)


@pytest.mark.gpu
@pytest.mark.parametrize("arch", ["intrinsics_unet", "ray_film_unet"])
def test_cli_trains_film_models(train_bin, tmp_path, arch):
    """The config-3 networks through build/train (TensorBoardTrainerEnhanced: camera from each batch's
    K, FiLM forward, per-sample validation) with their torch::save checkpoints."""
    cfg = yaml.safe_load(open(os.path.join(ROOT, "configs", "train_config.yaml")))
    cfg["data"].update(dataset_name="synthetic", num_train_samples=8, num_val_samples=3, input_height=48,
                       input_width=64)
    cfg["model"].update(architecture=arch, init_features=8)
    cfg["training"].update(num_epochs=2, batch_size=4, val_interval=1)
    cfg["checkpointing"].update(checkpoint_dir=str(tmp_path / "ckpt"), save_interval=1)
    cfg["logging"]["log_dir"] = str(tmp_path / "logs")
    p = tmp_path / "cfg.yaml"
    p.write_text(yaml.safe_dump(cfg))
    r = subprocess.run([train_bin, "-c", str(p)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert f"Model: {arch}" in r.stdout
    rows = (tmp_path / "logs" / "baseline_unet" / "metrics.csv").read_text().strip().splitlines()
    assert [row.split(",")[:2] for row in rows[1:]] == [["1", "0"], ["2", "2"]]
    vals = [float(x) for x in rows[-1].split(",")[2:5]]
    assert all(v == v and v > 0 for v in vals)
    import torch
    sd = torch.jit.load(str(tmp_path / "ckpt" / "baseline_unet" / "baseline_unet_epoch_2.pt")).state_dict()
    assert "enc1.film.fc1.weight" in sd and int(sd["enc1.film.bn1.num_batches_tracked"]) == 4
    if arch == "ray_film_unet":
        assert tuple(sd["enc1.conv1.weight"].shape) == (8, 6, 3, 3)   # rgb + rays
    tb = (tmp_path / "logs" / "baseline_unet" / "tensorboard_scalars.csv").read_text()
    assert "loss_components/reproj_loss,2," in tb and "metrics/abs_rel,2," in tb


@pytest.mark.gpu
@pytest.mark.parametrize("variant,pcl,att", [("full", True, True), ("lightweight", True, True), ("full", False, False)])
def test_cli_trains_geometry_aware(train_bin, tmp_path, variant, pcl, att):
    """model.architecture: geometry_aware (train_config.yaml:44-57 and its geometry_aware_full /
    _lightweight / ablation_rays_only experiments) through build/train: GeometryTrainer over
    GeometryAwareNetworkImpl / LightweightGeometryNetworkImpl, per-sample validation, metrics.csv,
    .cadckpt checkpoints."""
    cfg = yaml.safe_load(open(os.path.join(ROOT, "configs", "train_config.yaml")))
    cfg["data"].update(dataset_name="synthetic", num_train_samples=8, num_val_samples=3, input_height=64,
                       input_width=64)
    cfg["model"].update(architecture="geometry_aware", variant=variant, use_pcl=pcl, use_attention=att,
                        init_features=8)
    cfg["training"].update(num_epochs=2, batch_size=4, val_interval=1)
    cfg["checkpointing"].update(checkpoint_dir=str(tmp_path / "ckpt"), save_interval=1)
    cfg["logging"]["log_dir"] = str(tmp_path / "logs")
    p = tmp_path / "cfg.yaml"
    p.write_text(yaml.safe_dump(cfg))
    r = subprocess.run([train_bin, "-c", str(p)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert f"Model: geometry_aware/{variant}" in r.stdout
    rows = (tmp_path / "logs" / "baseline_unet" / "metrics.csv").read_text().strip().splitlines()
    assert [row.split(",")[:2] for row in rows[1:]] == [["1", "0"], ["2", "2"]]
    vals = [float(x) for x in rows[-1].split(",")[2:5]]
    assert all(v == v and v > 0 for v in vals)
    assert (tmp_path / "ckpt" / "baseline_unet" / "final_model.cadckpt").exists()
    assert (tmp_path / "ckpt" / "baseline_unet" / "baseline_unet_epoch_2.cadckpt").exists()


def test_cli_data_parallel_plan(train_bin, tmp_path, cad):
    """build/train's data-parallel plumbing on the CPU (--dry-run stops every rank before its first GPU
    call and stands in for the collective): hardware.num_gpus ranks are started as child processes,
    each bound to its gpu_ids entry; rank 0's communicator id reaches every rank through the
    rendezvous file; each rank trains its own B-slice of the global batch (last partial global batch
    dropped); the bucket plan is the library's (cad_plan_grad_buckets)."""
    p = _dp_cfg(tmp_path)
    r = subprocess.run([train_bin, "-c", str(p), "--dry-run"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    plans = sorted((json.loads(line) for line in r.stdout.strip().splitlines()), key=lambda d: d["rank"])
    assert [d["rank"] for d in plans] == [0, 1] and all(d["world"] == 2 and d["communicator"] for d in plans)
    assert [d["device"] for d in plans] == [3, 5]
    assert plans[0]["id_hash"] == plans[1]["id_hash"]
    assert [d["first_step_samples"] for d in plans] == [[0, 8], [8, 16]]
    assert all(d["steps_per_epoch"] == 100 // 16 and d["global_batch"] == 16 for d in plans)
    lib = cad.load_library()
    ns, off, cnt, nf = C.c_int(), (C.c_int64 * 16)(), (C.c_int64 * 16)(), C.c_int64()
    assert lib.cad_model_grad_layout(0, 3, 16, C.byref(ns), off, cnt, C.byref(nf)) == 0
    bo, bc, bl = (C.c_int64 * 16)(), (C.c_int64 * 16)(), (C.c_int * 16)()
    nb = lib.cad_plan_grad_buckets(off, cnt, ns.value, 25 << 18, bo, bc, bl)
    assert plans[0]["buckets"] == [[bo[i], bc[i], bl[i]] for i in range(nb)] == plans[1]["buckets"]
    assert plans[0]["n_flat"] == nf.value


def test_cli_data_parallel_single_process_and_errors(train_bin, tmp_path):
    # one GPU with distributed: true -> one process with a single-rank communicator
    p = _dp_cfg(tmp_path, num_gpus=1, gpu_ids=[2])
    r = subprocess.run([train_bin, "-c", str(p), "--dry-run"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip())
    assert (d["rank"], d["world"], d["device"], d["communicator"], d["steps_per_epoch"]) == (0, 1, 2, True, 13)
    # distributed: false ignores num_gpus (the reference's default), no communicator
    p = _dp_cfg(tmp_path, distributed=False)
    d = json.loads(subprocess.run([train_bin, "-c", str(p), "--dry-run"], capture_output=True, text=True,
                                  timeout=60).stdout.strip())
    assert (d["world"], d["communicator"]) == (1, False)
    # the gradient exchange is RCCL: another backend is refused with the reference's error contract
    p = _dp_cfg(tmp_path, backend="gloo")
    r = subprocess.run([train_bin, "-c", str(p), "--dry-run"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and r.stderr.startswith("Error: hardware.backend")


@pytest.mark.gpu
def test_cli_distributed_single_rank_matches_plain(train_bin, tmp_path):
    """distributed: true on one GPU runs the RCCL path (communicator, parameter broadcast, bucketed
    all-reduce overlapped with the backward, loss all-reduce) on a single-rank communicator: the
    trajectory must equal the plain single-process run bit for bit."""
    rows = {}
    for dist in (False, True):
        cfg = yaml.safe_load(open(os.path.join(ROOT, "configs", "train_config.yaml")))
        cfg["data"].update(dataset_name="synthetic", num_train_samples=16, num_val_samples=8, input_height=64,
                           input_width=64)
        cfg["training"].update(num_epochs=2, batch_size=8)
        cfg["checkpointing"]["checkpoint_dir"] = str(tmp_path / f"ckpt{dist}")
        cfg["logging"]["log_dir"] = str(tmp_path / f"logs{dist}")
        cfg["hardware"] = {"device": "cuda", "gpu_ids": [0], "num_gpus": 1, "distributed": dist, "backend": "nccl"}
        p = tmp_path / f"cfg{dist}.yaml"
        p.write_text(yaml.safe_dump(cfg))
        r = subprocess.run([train_bin, "-c", str(p)], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        assert ("RCCL" in r.stdout) == dist
        csv = (tmp_path / f"logs{dist}" / "baseline_unet" / "metrics.csv").read_text().strip().splitlines()
        rows[dist] = [line.split(",")[:11] for line in csv[1:]]   # all but learning_rate, time
    assert rows[True] == rows[False]


def _manifest_tree(tmp_path, n=6, rgb_ext=".png"):
    """n samples (RGB frames PNG or JPEG, depth PNG) under tmp_path (paths in the manifest relative to
    it, the run's cwd)."""
    import numpy as np
    from PIL import Image
    rng = np.random.default_rng(0)
    images = []
    for k in range(n):
        rel = f"./data/sunrgbd/SUNRGBD/kv1/NYUdata/NYU{k:04d}"
        d = tmp_path / rel
        (d / "image").mkdir(parents=True)
        (d / "depth").mkdir(parents=True)
        Image.fromarray(rng.integers(0, 256, (60, 80, 3), dtype=np.uint8)).save(d / "image" / ("rgb" + rgb_ext))
        Image.fromarray(rng.integers(500, 9000, (60, 80), dtype=np.uint16)).save(d / "depth" / "depth.png")
        (d / "intrinsics.txt").write_text("518.8 0 325.5\n0 519.4 253.7\n0 0 1\n")
        images.append({"path": rel, "sensor_type": "kv1", "valid": True})
    (tmp_path / "manifest.json").write_text(json.dumps({"dataset": "SUN RGB-D V1", "images": images}))


def test_cli_manifest_dataset_plan(train_bin, tmp_path):
    """data.dataset_name sunrgbd: the sample count comes from the manifest (read on the host, before
    any GPU call), validation takes min(500, size) of the same samples."""
    pytest.importorskip("PIL")
    _manifest_tree(tmp_path, 7)
    cfg = {"data": {"dataset_name": "sunrgbd", "manifest_path": "./manifest.json", "input_height": 48,
                    "input_width": 64},
           "model": {"init_features": 16}, "training": {"batch_size": 2, "num_epochs": 1}}
    p = tmp_path / "m.yaml"
    p.write_text(yaml.safe_dump(cfg))
    r = subprocess.run([train_bin, "-c", str(p), "--dry-run"], capture_output=True, text=True, timeout=60,
                       cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip())["steps_per_epoch"] == 4   # 7 samples, batch 2, last partial kept
    cfg["data"]["manifest_path"] = "./missing.json"
    p.write_text(yaml.safe_dump(cfg))
    r = subprocess.run([train_bin, "-c", str(p), "--dry-run"], capture_output=True, text=True, timeout=60,
                       cwd=tmp_path)
    assert r.returncode == 1 and "Cannot open manifest file" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("rgb_ext", [".png", ".jpg"])
def test_cli_trains_from_manifest(train_bin, tmp_path, rgb_ext):
    """build/train on SUN RGB-D manifest samples (PNG, or JPEG RGB frames as SUN RGB-D ships them)
    through the prefetch ring (decode threads, pinned upload, device resize + augmentation)."""
    _manifest_tree(tmp_path, 6, rgb_ext)
    cfg = yaml.safe_load(open(os.path.join(ROOT, "configs", "train_config.yaml")))
    cfg["data"].update(dataset_name="sunrgbd", manifest_path="./manifest.json", input_height=48, input_width=64)
    cfg["model"]["init_features"] = 16
    cfg["training"].update(num_epochs=2, batch_size=4)
    cfg["checkpointing"]["checkpoint_dir"] = str(tmp_path / "ckpt")
    cfg["logging"]["log_dir"] = str(tmp_path / "logs")
    p = tmp_path / "cfg.yaml"
    p.write_text(yaml.safe_dump(cfg))
    r = subprocess.run([train_bin, "-c", str(p)], capture_output=True, text=True, timeout=300, cwd=tmp_path)
    assert r.returncode == 0, r.stderr
    assert "Training samples: 6 (./manifest.json)" in r.stdout
    rows = (tmp_path / "logs" / "baseline_unet" / "metrics.csv").read_text().strip().splitlines()
    assert len(rows) == 3 and rows[-1].startswith("2,2,")   # 2 steps per epoch (4 + 2 samples)
    vals = [float(x) for x in rows[-1].split(",")[2:5]]
    assert all(v == v and v > 0 for v in vals)   # finite train loss, val loss, abs_rel

"""The N>1 path of bench.py (the driver's 1/2/4/8-GPU scaling runs launch it as
`torch.distributed.run --nproc-per-node N ... bench.py --gpus N`), rehearsed before a driver run is its
first execution:

  * CPU (gloo, world 2): the launcher plumbing — setup_dist reads RANK / WORLD_SIZE / LOCAL_RANK and
    joins the gloo store, and rank 0's 128-byte RCCL unique id (cad_comm_get_unique_id, a host-side
    bootstrap call) reaches every rank intact through it (bench.rccl_unique_id), as the RCCL
    communicator of --exchange rccl needs;
  * GPU: the whole bench under torch.distributed.run with 2 ranks sharing the one GPU of the box
    (CAD_BENCH_DEVICE=0; --exchange torch over gloo, since RCCL refuses two ranks on one device),
    tiny shapes: rank 0 prints one JSON line with n_gpus 2, dp2 and the max-over-ranks clock."""
import json
import os
import socket
import subprocess
import sys
import types

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _uid_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    os.environ.pop("CAD_BENCH_DEVICE", None)
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    import bench
    import cad_pkg
    cad = cad_pkg.load()
    w, r, local = bench.setup_dist(types.SimpleNamespace(gpus=world))
    uid = bench.rccl_unique_id(cad, r)
    q.put((rank, w, r, local, uid))
    dist.barrier()
    dist.destroy_process_group()


def test_rccl_unique_id_handoff_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_uid_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, w0, rr0, l0, u0), (r1, w1, rr1, l1, u1) = got
    assert (w0, w1) == (2, 2) and (rr0, rr1) == (0, 1) and (l0, l1) == (0, 1)
    assert len(u0) == 128 and u0 == u1 and any(u0)


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bench_two_ranks_one_gpu():
    env = dict(os.environ, CAD_BENCH_DEVICE="0", CAD_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--exchange", "torch", "--steps", "2", "--warmup", "1", "--batch", "2", "--height", "64",
           "--width", "64", "--features", "8", "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]   # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 4
    assert out["value"] > 0 and out["ms_per_step"] > 0 and out["scaling"] == "weak"
    assert "torch.distributed" in out["config"]["gradient_exchange"]
    assert out["last_loss"] == out["last_loss"]   # finite
    # exchange accounting of the timed steps (what the driver's first multi-GPU run reports)
    n_flat = out["config"]["params"]
    x = out["exchange"]
    assert x["comm_size"] == 2 and x["steps_accounted"] == 2 and "torch.distributed" in x["backend"]
    assert x["allreduces_per_step"] >= 1 and x["bytes_allreduced_per_step"] >= 4 * n_flat
    assert x["exposed_ms_per_step_rank0"] is not None and x["exposed_ms_per_step_rank0"] >= 0
    assert x["exposed_ms_per_step_max_rank"] >= x["exposed_ms_per_step_rank0"] - 1e-9
    # the DP workloads BASELINE names for N > 1 (configs[3], configs[4] bf16 and MXFP8), same exchange
    legs = out["dp_workloads"]
    assert set(legs) == {"config4", "config5", "config5_fp8"}
    for key, leg in legs.items():
        assert "error" not in leg, (key, leg)
        assert leg["n_gpus"] == 2 and leg["value"] > 0 and leg["last_loss"] == leg["last_loss"]
        assert leg["exchange"]["comm_size"] == 2 and leg["exchange"]["steps_accounted"] == leg["steps"]
        assert leg["exchange"]["bytes_allreduced_per_step"] > 0

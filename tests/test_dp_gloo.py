"""Data-parallel path on CPU with the gloo backend (world_size 2): the decoder-first bucketed
all-reduce of the Trainer (GradBucketer) reduces every gradient element exactly once, whatever the
bucket size, and DP semantics (per-replica loss/BN, mean gradient, global clip,
replicated Adam) equal the oracle's single-process emulation."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# stage ranges like the U-Net's: contiguous, decreasing offsets (head last in the slab)
STAGES = [(960, 40), (700, 260), (500, 200), (300, 200), (250, 50), (100, 150), (60, 40), (30, 30), (8, 22), (0, 8)]
N_FLAT = 1000


def _bucket_worker(rank, world, port, bucket_elems, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, ROOT)
    import cad_pkg
    cad_pkg.load()
    from cad_amd.model import GradBucketer
    flat = torch.zeros(N_FLAT)
    bk = GradBucketer(flat, len(STAGES), bucket_elems, None)
    for s, (off, cnt) in enumerate(STAGES):
        flat[off:off + cnt] = (rank + 1) * (s + 1) + torch.arange(cnt, dtype=torch.float32) * 0.5
        bk.on_stage(s, off, cnt)
    bk.wait()
    expect = torch.zeros(N_FLAT)
    for s, (off, cnt) in enumerate(STAGES):
        expect[off:off + cnt] = sum((r + 1) * (s + 1) for r in range(world)) + world * torch.arange(cnt) * 0.5
    ok = torch.equal(flat, expect)
    covered = sorted(bk.buckets)
    contiguous = covered[0][0] == 0 and covered[-1][1] == N_FLAT and all(
        a[1] == b[0] for a, b in zip(covered, covered[1:]))
    q.put((rank, ok, contiguous, len(bk.buckets)))
    dist.destroy_process_group()


@pytest.mark.parametrize("bucket_elems", [1, 300, 10_000])
def test_bucketed_allreduce_gloo(bucket_elems):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bucket_worker, args=(r, 2, port, bucket_elems, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok and cont for _, ok, cont, _ in res), res
    nb = {n for *_, n in res}
    assert len(nb) == 1
    if bucket_elems == 1:
        assert nb == {len(STAGES)}
    if bucket_elems == 10_000:
        assert nb == {1}


def _dp_oracle_worker(rank, world, port, q):
    """Each rank runs the oracle step on its own shard with the gradient mean taken by all-reduce —
    the DP semantics of cad_amd.Trainer; compared against the single-process emulation."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, ROOT)
    torch.set_num_threads(2)
    from oracle import cad_oracle as O
    f, B, H, W = 4, 2, 32, 32
    params, bufs = O.init_params(f, seed=3), O.init_buffers(f)
    rgb, gt, K = [torch.from_numpy(a) for a in O.synth_batch(B * world, H, W)]
    sl = slice(rank * B, (rank + 1) * B)
    tr = O.Trainer(params, bufs)
    _, _, _, _, grads = tr.forward_backward(rgb[sl], gt[sl], K[sl])
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat)
    flat /= world
    out, o = [], 0
    for g in grads:
        out.append(flat[o:o + g.numel()].view_as(g).clone())
        o += g.numel()
    tr.apply(out)
    q.put((rank, torch.cat([p.reshape(-1) for p in tr.p.values()])))
    dist.destroy_process_group()


def test_dp_semantics_gloo(oracle):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_oracle_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    # replicas stay identical
    assert torch.equal(res[0], res[1])
    # single-process emulation: per-shard grads, mean, global clip, Adam
    f, B, H, W = 4, 2, 32, 32
    params, bufs = oracle.init_params(f, seed=3), oracle.init_buffers(f)
    rgb, gt, K = [torch.from_numpy(a) for a in oracle.synth_batch(B * world, H, W)]
    shard_grads = []
    for r in range(world):
        t = oracle.Trainer(params, bufs)
        shard_grads.append(t.forward_backward(rgb[r * B:(r + 1) * B], gt[r * B:(r + 1) * B], K[r * B:(r + 1) * B])[4])
    mean = [sum(gs) / world for gs in zip(*shard_grads)]
    t = oracle.Trainer(params, bufs)
    t.apply(mean)
    ref = torch.cat([p.reshape(-1) for p in t.p.values()])
    assert (ref - res[0]).abs().max().item() < 1e-6

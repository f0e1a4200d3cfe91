"""N > 1 path on CPU with gloo, world size 2 (the GPU run uses RCCL): segments
are sharded contiguously with no data-path collective; timing is reduced with
max over ranks; the union of the shards is the whole batch."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from uplink_amd.shard import max_over_ranks, min_over_ranks, segment_seed, shard_range


def test_shard_range_covers_exactly_once():
    for total in (0, 1, 7, 1024):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                s, c = shard_range(total, world, r)
                seen += list(range(s, s + c))
            assert seen == list(range(total))
    assert shard_range(1024, 8, 3) == (384, 128)  # C4: 128 segments per GPU


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    k, n, ess, stripes, total = 4, 10, 64, 3, 5
    f = O.FEC(k, n)
    start, count = shard_range(total, world, rank)
    out = {}
    for g in range(start, start + count):
        seg = np.random.default_rng(segment_seed(g)).integers(0, 256, stripes * k * ess, dtype=np.uint8)
        out[g] = f.encode_segment(seg, ess)
    t = max_over_ranks(float(rank + 1))
    ok = min_over_ranks(1)
    q.put((rank, {g: v.tobytes() for g, v in out.items()}, t, ok))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_sharded_encode(oracle):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in procs]
    res = [q.get(timeout=120) for _ in range(world)]
    [p.join(timeout=60) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    merged = {}
    for rank, d, t, ok in res:
        assert t == float(world)  # max over ranks
        assert ok == 1
        assert not (set(d) & set(merged))  # no segment processed twice
        merged.update(d)
    assert sorted(merged) == list(range(5))
    f = oracle.FEC(4, 10)
    for g, v in merged.items():
        seg = np.random.default_rng(segment_seed(g)).integers(0, 256, 3 * 4 * 64, dtype=np.uint8)
        assert v == f.encode_segment(seg, 64).tobytes()


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_bench_two_ranks_hip_path_gloo_on_one_gpu():
    """The bench's N > 1 path with the HIP engine: two ranks (torch
    distributed run) share the box's one GPU and use gloo for the barrier and
    the max over ranks; each rank encodes and rebuilds its own contiguous
    shard of 64 segments (32 each) with no data-path collective, and the
    rank-0 line reports the whole job.  The driver's multi-GPU runs use RCCL
    (the default backend) on one GPU per rank."""
    import json
    import subprocess
    import sys
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, BENCH_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"), "--gpus", "2", "--steps",
           "2", "--warmup", "1", "--settle-s", "0", "--total-segments", "64", "--cpu-sample-s", "0.5",
           "--no-other-configs"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, env=env, cwd=root)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["verified"] is True
    assert line["config"]["total_segments_per_step"] == 64 and line["config"]["segments_this_rank"] == 32
    assert line["value"] > 0
    # the record shows that both ranks took part, and each rank's own wall time
    assert line["ranks_seen"] == 2
    assert len(line["rank_wall_s"]) == 2 and all(w > 0 for w in line["rank_wall_s"])
    assert line["ms_per_step"] == pytest.approx(max(line["rank_wall_s"]) / line["steps"] * 1e3, rel=1e-3)
    # the N > 1 line carries the same-run CPU baseline and the fresh-share-set decode leg
    assert line["cpu_baseline"]["value"] > 0 and line["cpu_baseline"]["cores"] >= 1
    fs = line["fresh_share_sets"]
    assert fs["32 segments, 32 fresh seeded 29-subsets per launch"]["verified"] is True
    assert fs["one segment, fresh set"]["wall_us_median"] > 0
    # the timed decode is the share-set pass (fresh sets), the warm shared-set
    # decode and the encoder's no-arithmetic schedule are reported beside it
    assert line["kernels"]["decode"]["kernel"].startswith("rs_sets_prep")
    assert line["kernels"]["decode_warm_shared_set"]["verified"] is True
    assert line["roofline"]["encode_shape_GBps_on_box"] > 0 and line["roofline"]["frac_of_shape"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(420)
def test_bench_configs3_eight_ranks_on_one_gpu():
    """BASELINE configs[3] as the driver's 8-GPU run shards it: 1024 RS(29,80)
    64 MiB segments per step, 128 per rank, contiguous shards, no data-path
    collective.  Here all eight ranks share the box's one GPU (gloo for the
    barrier and the max over ranks; the driver's run uses RCCL, one GPU per
    rank); every rank encodes and rebuilds its own 128 segments and checks
    them, and the rank-0 line reports the whole job."""
    import json
    import subprocess
    import sys
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, BENCH_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"), "--gpus", "8", "--steps",
           "1", "--warmup", "1", "--settle-s", "0", "--no-cpu-baseline", "--no-other-configs",
           "--batch", "16"]  # eight ranks' pools on one GPU: 2 x 16 segments each
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd=root)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 8 and line["verified"] is True
    assert line["config"]["total_segments_per_step"] == 1024 and line["config"]["segments_this_rank"] == 128
    assert line["ranks_seen"] == 8 and len(line["rank_wall_s"]) == 8
    assert line["value"] > 0


@pytest.mark.gpu
def test_bench_rccl_branch_at_world_one():
    """the RCCL branch the driver's 8-GPU run takes --
    init_process_group("nccl", device_id=...), the barriers, the device-tensor
    all_gather of the wall times and the all_reduce of the rank count and the
    verification flag -- run here on one GPU: bench.py under torch.distributed.run
    with one rank and BENCH_FORCE_DIST=1 (no BENCH_DIST_BACKEND: RCCL)."""
    import json
    import subprocess
    import sys
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, BENCH_FORCE_DIST="1")
    env.pop("BENCH_DIST_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"), "--gpus", "1", "--steps",
           "2", "--warmup", "1", "--settle-s", "0", "--total-segments", "32", "--no-cpu-baseline",
           "--no-other-configs"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, env=env, cwd=root)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["collectives"] == "nccl"
    assert line["n_gpus"] == 1 and line["verified"] is True
    assert line["ranks_seen"] == 1 and len(line["rank_wall_s"]) == 1
    assert line["config"]["segments_this_rank"] == 32

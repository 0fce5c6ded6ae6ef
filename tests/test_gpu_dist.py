"""ShardedProjector itself on the GPU with 2 ranks (child processes sharing cuda:0 over gloo):
R built on rank 0 only and broadcast, each rank projecting only its own rows — a host shard, a
device shard, and its byte split of a libsvm file written to Parquet part files — and the pieces
assembling to the oracle's product of the whole matrix (code/clustermode/randomProjection.py:
72,104,107-113)."""
import glob
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import scipy.sparse as sp

from oracle import smmp
from oracle.libsvm_ref import parse_text
from randomprojection_amd import egress, srp_matrix as sm

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_sharded_projector_two_ranks(tmp_path):
    world = 2
    rng = np.random.default_rng(8)
    m = 300_000
    lines = []
    for i in range(3000):
        idx = np.sort(rng.choice(m, int(rng.integers(0, 20)), replace=False)) + 1
        lines.append(f"{i % 2}" + "".join(f" {j}:{rng.standard_normal():.6g}" for j in idx))
    text = ("\n".join(lines) + "\n").encode()
    tp = tmp_path / "train.libsvm"
    tp.write_bytes(text)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), WORLD_SIZE=str(world))
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_gpu_worker.py"), str(tmp_path), str(tp)],
                              env=dict(env, RANK=str(r), LOCAL_RANK="0"), stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(world)]
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=240)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert all(p.returncode == 0 for p in procs), "\n".join(o[-3000:] for o in outs)
    res = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    A = sp.csr_matrix((res[0]["A_data"], res[0]["A_indices"], res[0]["A_indptr"]), shape=(res[0]["A_indptr"].size - 1, m))
    R = sm.projection_operand(sm.sparse_random_matrix(256, m, random_state=123))
    Wp, Wj, Wx, _, _ = smmp.matmat(A, R)
    for pre in ("", "d_"):
        gp, gj, gx = [0], [], []
        for r in range(world):
            z = res[r]
            assert int(z[pre + "row" if pre else "row_off"]) == len(gp) - 1
            assert int(z[pre + "nnz" if pre else "nnz_off"]) == len(gj)
            ip = z[pre + "indptr"].astype(np.int64)
            gp.extend((len(gj) + ip[1:] - ip[0]).tolist())
            gj.extend(z[pre + "indices"].tolist())
            gx.append(z[pre + "data"])
        assert np.array_equal(np.array(gp), Wp) and np.array_equal(np.array(gj), Wj)
        assert np.array_equal(np.concatenate(gx).view(np.uint32), Wx.view(np.uint32))
    # libsvm splits: each rank's part files; together every line once, ids unique and increasing
    assert res[0]["byte_range"][1] == res[1]["byte_range"][0]
    files = sorted(glob.glob(str(tmp_path / "parquet" / "part-*.parquet")))
    assert sorted(files) == sorted(str(f) for z in res for f in z["parts"])
    ids, labels, Cs = [], [], []
    for f in files:
        i_, l_, c_ = egress.read_parquet(f)
        ids.append(i_)
        labels.append(l_)
        Cs.append(c_)
    ids = np.concatenate(ids)
    assert np.all(np.diff(ids) > 0) and ids.size == 3000
    assert (ids[-1] >> 33) >= (1 << 20)  # rank 1's partitions
    lab, ip, ij, iv = parse_text(text, m)
    X = sp.csr_matrix((iv, ij, ip), shape=(lab.size, m))
    Xp, Xj, Xx, _, _ = smmp.matmat(X, R)
    Xj, Xx = smmp.sorted_rows(Xp, Xj, Xx)
    C = sp.vstack(Cs).tocsr()
    assert np.array_equal(np.concatenate(labels), lab.astype(np.float32))
    assert np.array_equal(C.indptr, Xp) and np.array_equal(C.indices, Xj)
    assert np.array_equal(C.data, Xx.astype(np.float64))


def test_bench_host_boundary_two_ranks():
    """bench.py --boundary host at N = 2 (rehearsed with both ranks on cuda:0 over gloo): every rank
    streams its own host shard through rp_project_stream, the wall time is the max over ranks, and
    every rank's sampled rows equal the oracle's (the N = 8 driver path is the same code over RCCL)."""
    import json

    world = 2
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), WORLD_SIZE=str(world),
               RP_BENCH_REHEARSE_ONE_GPU="1")
    bench = os.path.join(os.path.dirname(HERE), "bench.py")
    args = [sys.executable, bench, "--boundary", "host", "--rows", "3000000", "--m", "2000000", "--steps", "2",
            "--warmup", "1", "--chunk-rows", "1000000"]
    procs = [subprocess.Popen(args, env=dict(env, RANK=str(r), LOCAL_RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(world)]
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=240))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert all(p.returncode == 0 for p in procs), "\n".join(o[1][-3000:] for o in outs)
    line = json.loads([ln for ln in outs[0][0].splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["boundary"] == "host"
    assert line["verified"]["sample_bitexact_vs_oracle"] and line["verified"]["indptr_ok"]
    assert line["value"] > 0 and not [ln for ln in outs[1][0].splitlines() if ln.startswith("{")]


def test_bench_gpus_two_launches_two_ranks():
    """`bench.py --gpus 2` with no launcher starts its own 2 ranks (rehearsed on cuda:0 over gloo on
    this one-GPU box; the driver's 8-GPU node runs the same code over RCCL): the line reports
    n_gpus == ranks_seen == 2, every rank's sampled rows are bit-exact against the oracle, and rank
    0's host CPU baseline is still there at N > 1 (code/clustermode/randomProjection.py:104,107-110)."""
    import json

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["RP_BENCH_REHEARSE_ONE_GPU"] = "1"
    bench = os.path.join(os.path.dirname(HERE), "bench.py")
    r = subprocess.run([sys.executable, bench, "--gpus", "2", "--rows", "2000000", "--m", "3000000", "--steps", "2",
                        "--warmup", "1", "--cpu-sample-rows", "200000", "--cpu-part-rows", "20000"],
                       env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["ranks_seen"] == 2 and line["backend"] == "gloo"
    v = line["verified"]
    assert v["sample_bitexact_vs_oracle"] and v["indptr_ok"] and v["columns_ok"] and v["ranks_verified"] == 2
    assert line["cpu_baseline"] and line["cpu_baseline"]["value"] > 0
    assert line["librp"]["checked_against_sources"] and line["value"] > 0
    # boundary 2 beside it: every rank streams its own rows host CSR -> host CSR, checked after the clock
    h = line["boundaries"]["host"]
    assert h["rows_per_s"] > 0 and h["verified"]["sample_bitexact_vs_oracle"] and h["verified"]["indptr_ok"]
    assert h["verified"]["nnz_out_equal_device_leg"]


def test_bench_rccl_path_one_rank():
    """The RCCL branch of bench.py executes on this one-GPU box (RP_BENCH_FORCE_PG=1 at world size 1):
    init_process_group("nccl", device_id=...), the broadcast of R's packed device image over RCCL,
    the projector rebuilt from the received image (rp_projector_create_from_device), barriers, and
    the projection by that projector checked against the oracle — the code the 8-GPU driver run uses,
    minus the peers."""
    import json

    env = {k: v for k, v in os.environ.items() if k not in ("RP_BENCH_REHEARSE_ONE_GPU",)}
    env.update(RP_BENCH_FORCE_PG="1", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_port()))
    bench = os.path.join(os.path.dirname(HERE), "bench.py")
    r = subprocess.run([sys.executable, bench, "--gpus", "1", "--rows", "1000000", "--m", "3000000", "--steps", "2",
                        "--warmup", "1", "--no-cpu-baseline"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["backend"] == "nccl" and line["ranks_seen"] == 1 and line["r_from_broadcast_image"]
    assert line["verified"]["sample_bitexact_vs_oracle"] and line["verified"]["indptr_ok"]

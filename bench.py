"""Benchmark: rows/s projected (KDD2012 54,686,452 -> 4096, R from SparseRandomProjection(random_state=123)).

One step = one pass of the hot path (C = A @ R: one rp_project_device call, i.e. every kernel of the
pipeline it runs) over the whole workload, inputs resident in HBM when timing starts
(boundary 1 of SURVEY.md §8(d)); --boundary host / libsvm time boundaries 2 and 3 instead:
  N=1: BASELINE.json configs[1] — the full KDD2012 train shape, 119,705,032 synthetic rows
       (per-row nnz 1 + Poisson(10), distinct uniform columns, values 1.0) on one MI355X.
  N>1: weak scaling — every rank projects its own 119,705,032-row shard (configs[2]'s
       row-sharding), R packed once on rank 0 and broadcast over RCCL; no collective in the loop.
  --config kdd9x: configs[2] itself, 1,077,345,288 rows split over the ranks (strong scaling);
  --config cfg4: configs[3], 200M x 10M power-law rows with exactly 100 nnz -> 1024.
Prints ONE JSON line on rank 0 (see DESIGN.md §5 for every field).

    python bench.py [--config kdd|kdd9x|cfg4] [--gpus N] [--steps K] [--warmup W] [--rows R]
                    [--boundary device|host|libsvm]

--gpus N with N > 1 and no WORLD_SIZE in the environment: this process makes no GPU call, starts
N rank processes of itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / a free
MASTER_PORT, as torch.distributed.run sets them), relays rank 0's line and exits with the worst
rank's status. Under torch.distributed.run (WORLD_SIZE set) a --gpus that differs from WORLD_SIZE
is an error, never a silent 1-GPU line.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
PCIE_PEAK_GBS = 63.0  # PCIe Gen5 x16 per direction (measured copies: H2D ~55 GB/s, scripts/probes/pcie_probe2.hip)
RANDOM_LINE_CEILING = 55e9  # random 128-B line fills/s, measured (scripts/probes/gather_probe*.hip)


# BASELINE.json configs: [1] KDD2012 train on one GPU (the headline); [3] the power-law stress shape
CONFIGS = {
    "kdd": {"rows": 119_705_032, "m": 54_686_452, "p": 4096, "dist": "uniform", "mean_extra": 10.0,
            "cpu_sample_rows": 32_000_000,
            "metric": "rows/sec projected (whole node), KDD2012 54.7M->4096 dims; achieved HBM GB/s",
            "workload": "configs[1]: KDD2012 train {rows} rows x {m} -> {p} per GPU, device-resident CSR in/out",
            "data": "synthetic KDD2012-shaped rows ({dist} columns, 1+Poisson(10) nnz/row, values 1.0), "
                    "R = SparseRandomProjection({p}, random_state=123) regenerated bit-identically"},
    "kdd9x": {"rows": 1_077_345_288, "m": 54_686_452, "p": 4096, "dist": "uniform", "mean_extra": 10.0,
              "cpu_sample_rows": 64_000_000, "strong": True,
              "metric": "rows/sec projected (whole node), KDD2012 54.7M->4096 dims; achieved HBM GB/s",
              "workload": "configs[2]: 9x KDD2012 train, 1,077,345,288 rows x {m} -> {p} row-sharded over the "
                          "ranks ({rows} on this rank), device-resident CSR in/out",
              "data": "synthetic KDD2012-shaped rows ({dist} columns, 1+Poisson(10) nnz/row, values 1.0), "
                      "R = SparseRandomProjection({p}, random_state=123) regenerated bit-identically"},
    "cfg4": {"rows": 200_000_000, "m": 10_000_000, "p": 1024, "dist": "powerlaw", "mean_extra": -100.0,
             "cpu_sample_rows": 4_000_000,
             "metric": "rows/sec projected, synthetic power-law 200M x 10M (100 nnz/row) -> 1024; achieved HBM GB/s",
             "workload": "configs[3]: power-law {rows} rows x {m}, 100 nnz/row -> {p} per GPU, device-resident CSR in/out",
             "data": "synthetic power-law rows ({dist} columns: Zipf(1.1) over a fixed permutation, exactly 100 "
                     "distinct nnz/row, values 1.0), R = SparseRandomProjection({p}, random_state=123)"},
}


LIB_ID, LIB_CHECKED = None, False  # build id of the loaded librp (keys profiles/*traffic*.json)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def launch_ranks(n: int) -> int:
    """--gpus N without a launcher: N child processes of this script, one per GPU (this process
    touches no GPU, so no exec/fork hazard), the torch.distributed.run environment set for each;
    rank 0's JSON line is relayed on stdout. A failing rank stops the others (their exact PIDs)."""
    import socket
    import subprocess

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n),
               LOCAL_WORLD_SIZE=str(n))
    procs = []
    for r in range(n):
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]],
                                      env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr, text=True))
    out0 = procs[0].communicate()[0]
    rcs = [procs[0].returncode]
    for q in procs[1:]:
        if rcs[0] != 0 and q.poll() is None:
            q.kill()
        rcs.append(q.wait())
    for ln in out0.splitlines():
        print(ln, flush=True)
    bad = [rc for rc in rcs if rc != 0]
    if bad:
        log(f"bench: rank exit codes {rcs}")
    return bad[0] if bad else 0


def step_kernels(plan, staged_run, call="sync"):
    """The kernels one rp_project_device call runs for this plan (rp_spgemm.hip). In auto mode a
    sync call has the host read lpr_choose_kernel's verdict and launch only the chosen branch; an
    async one launches the staged branch, gated on the device by the verdict."""
    if plan["pipeline"] == "rowlane":
        staged_kernels = staged_run or (call == "async" and plan["staged"] == "auto")
        main = ["lpr_reserve_kernel", "lpr_partition_kernel", "lpr_gather_kernel",
                "lpr_wave_kernel"] if staged_kernels else ["lpr_main_flat_kernel"]
        ks = main + ["lpr_heavy_count_kernel", "lpr_scan_kernel", "lpr_copy_kernel", "lpr_heavy_write_kernel"]
        if plan["staged"] == "auto":
            ks = ["lpr_choose_kernel"] + ks
        return ks
    return ["spgemm_lookback_kernel", "lpr_scan_kernel", "tile_heavy_write_kernel", "slot_copy_kernel"]


def algorithmic_bytes_per_row(a, rbar, c):
    """Gustavson no-reuse model on the reference's formats (f32 values, int32
    indices, int32 row pointers): A ptr + idx/val, R ptr pair + gathered entries, C ptr + idx/val."""
    return (4 + 8 * a) + a * (8 + 8 * rbar) + (4 + 8 * c)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=["kdd", "kdd9x", "cfg4"], default="kdd",
                    help="kdd: BASELINE configs[1] (default, weak scaling: 119.7M rows per GPU); kdd9x: "
                         "configs[2], 1.08B rows split over the GPUs (strong scaling); cfg4: configs[3], "
                         "200M x 10M power-law rows, exactly 100 nnz/row -> 1024")
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (= ranks) of this node; default WORLD_SIZE or 1 (see the module doc)")
    ap.add_argument("--lib", default=None, help="A/B timing only: load this librp build instead of the "
                                                "package's (its build id is reported, the line says so)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=None)
    ap.add_argument("--m", type=int, default=None)
    ap.add_argument("--p", type=int, default=None)
    ap.add_argument("--dist", choices=["uniform", "powerlaw"], default=None)
    ap.add_argument("--order", choices=["scipy", "sorted"], default="scipy")
    ap.add_argument("--staging", choices=["auto", "on", "off"], default="auto")
    ap.add_argument("--stage-shift", type=int, default=0, help="2^shift features per staging bucket (0 = auto)")
    ap.add_argument("--pipeline", choices=["auto", "tile", "rowlane"], default="auto",
                    help="force a kernel pipeline where it can run (results identical; measurements)")
    ap.add_argument("--cpu-sample-rows", type=int, default=None)
    ap.add_argument("--cpu-part-rows", type=int, default=100_000,
                    help="rows per recipe partition (one per core) in the CPU baseline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--part-rows", type=int, default=1_000_000,
                    help="--boundary partition: rows of the partition handed to the drop-in per step")
    ap.add_argument("--recipe-sample-rows", type=int, default=50_000,
                    help="--boundary partition: rows of the same partition run through the recipe (CPU baseline)")
    ap.add_argument("--boundary", choices=["device", "host", "libsvm", "partition"], default="device",
                    help="device: inputs/outputs resident in HBM (the default line); host: host CSR in -> host "
                         "CSR out through the chunked stream path (rp_project_stream, PCIe-inclusive); libsvm: "
                         "libsvm text in host memory -> GPU parse + projection -> host CSR "
                         "(rp_libsvm_project_stream; default 20M rows); partition: the reference's own boundary, "
                         "random_project_mappartitions_function on a partition of Row dicts (SparseVector "
                         "features) -> (id, label, SparseVector) tuples")
    ap.add_argument("--chunk-bytes", type=int, default=64 << 20, help="--boundary libsvm: text bytes per chunk")
    ap.add_argument("--host-mem", choices=["pageable", "pinned"], default="pinned",
                    help="--boundary host: host arrays in pageable (numpy) or page-locked (rp_host_alloc) memory")
    ap.add_argument("--chunk-rows", type=int, default=0, help="--boundary host: rows per chunk (0 = library default)")
    ap.add_argument("--host-steps", type=int, default=None,
                    help="device line: timed passes of the boundary-2 leg (host CSR stream) on the same rows "
                         "after the device-resident measurement (default 3 for --config kdd, else 0 = skip)")
    ap.add_argument("--lpr-chunk-rows", type=int, default=None, help="row-lane rows per chunk (RP_OPT_CHUNK_ROWS)")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="projector option (Projector.set_option; A/B measurements, results identical), e.g. "
                         "fused_copy=0")
    ap.add_argument("--call", choices=["sync", "async"], default="sync",
                    help="sync: each step asks for the exact nnz (rp_project_device with total_nnz: the host "
                         "reads the staging verdict and launches only the chosen branch, then waits for the "
                         "result); async: total_nnz NULL (never waits on the host; the verdict gates the staged "
                         "kernels on the device)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"))
    args = ap.parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and (args.gpus or 1) > 1:
        sys.exit(launch_ranks(args.gpus))
    if env_world is not None and args.gpus is not None and int(env_world) != args.gpus:
        sys.exit(f"bench: --gpus {args.gpus} but WORLD_SIZE={env_world}: refusing to measure a different "
                 "number of GPUs than asked")
    args.gpus = int(env_world or 1)
    cfg = CONFIGS[args.config]
    if args.boundary == "libsvm" and args.rows is None:
        args.rows = 20_000_000  # ~5 GB of text in host memory per rank
    if args.boundary == "partition" and args.rows is None:
        args.rows = args.part_rows
    if args.host_steps is None:
        args.host_steps = 3 if args.config == "kdd" else 0
    for k in ("rows", "m", "p", "dist", "cpu_sample_rows"):
        if getattr(args, k) is None:
            setattr(args, k, cfg[k])

    import torch
    import torch.distributed as dist

    from randomprojection_amd import Projector, srp_matrix as sm, synth
    from randomprojection_amd import _native as nat

    nat.load(args.lib)  # the package's librp is checked against the sources on disk (build id)
    global LIB_ID, LIB_CHECKED
    LIB_ID, LIB_CHECKED = nat.build_id(), args.lib is None

    world = args.gpus
    rank = int(os.environ.get("RANK", "0"))
    total_rows_cfg = args.rows
    if cfg.get("strong"):  # a fixed total split over the ranks (contiguous shards)
        args.rows = args.rows // world + (1 if rank < args.rows % world else 0)
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N>1 path on a one-GPU box only: every rank on cuda:0 over gloo
    # (RCCL refuses two ranks on one device); the driver's multi-GPU runs use neither
    rehearse = os.environ.get("RP_BENCH_REHEARSE_ONE_GPU") == "1"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # RP_BENCH_FORCE_PG=1 at one rank: the process group, the RCCL broadcast of R's device image and
    # the projector built from the received image all run (evidence for the N > 1 path on a 1-GPU box)
    pg = world > 1 or os.environ.get("RP_BENCH_FORCE_PG") == "1"
    if pg:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    # ---- R: generated once on rank 0 (sklearn-identical), packed and uploaded, broadcast over RCCL
    t0 = time.perf_counter()
    R_host = None
    if rank == 0:
        comp = sm.sparse_random_matrix(args.p, args.m, random_state=123)
        R_host = sm.projection_operand(comp)
        del comp
        P = Projector(R_host, device=local)
        meta = {f: getattr(P.info, f) for f in ("m", "p", "nnz", "layout", "value_type", "magnitude",
                                                "block_shift", "n_buffers")}
        meta["buffer_bytes"] = list(P.info.buffer_bytes)
    else:
        meta = None
    t_r = time.perf_counter() - t0
    t_bcast = 0.0
    if pg:
        box = [meta]
        dist.broadcast_object_list(box, src=0)
        meta = box[0]
        bufs = [torch.empty(max(int(b), 1), dtype=torch.uint8, device=dev) for b in meta["buffer_bytes"][:meta["n_buffers"]]]
        if rank == 0:
            P.export_image([b.data_ptr() for b in bufs])
        torch.cuda.synchronize()
        tb = time.perf_counter()
        for b in bufs:
            dist.broadcast(b, src=0)          # the recipe's sc.broadcast(R), once, over xGMI
        torch.cuda.synchronize()
        t_bcast = time.perf_counter() - tb
        if rank != 0 or world == 1:  # (one rank: rank 0 projects with the received image too)
            info = nat.ProjectorInfo()
            for f in ("m", "p", "nnz", "layout", "value_type", "magnitude", "block_shift", "n_buffers"):
                setattr(info, f, meta[f])
            for i, b in enumerate(meta["buffer_bytes"]):
                info.buffer_bytes[i] = int(b)
            P = Projector.from_image(info, [b.data_ptr() for b in bufs], device=local)
        del bufs
    log(f"[rank {rank}] R ready: layout={P.layout} nnz={P.nnz} ({t_r:.1f}s build, {t_bcast*1e3:.1f} ms bcast)")

    # ---- A: this rank's synthetic shard, generated in HBM
    t0 = time.perf_counter()
    Ap, Aj, Ax = synth.kdd_rows_device(args.rows, args.m, seed=2012 + rank, dist=args.dist, device=local,
                                       mean_extra=cfg["mean_extra"])
    torch.cuda.synchronize()
    nnz_a = int(Aj.numel())
    log(f"[rank {rank}] A: {args.rows} rows, nnz={nnz_a} ({time.perf_counter() - t0:.1f}s)")

    if pg:
        ranks_seen = dist.get_world_size()
        if ranks_seen != world:
            raise RuntimeError(f"process group has {ranks_seen} ranks, --gpus {world}")
    args.dist_info = {"ranks_seen": dist.get_world_size() if pg else 1,
                      "backend": dist.get_backend() if pg else None,
                      "r_broadcast_ms": t_bcast * 1e3, "rehearsal_one_gpu": rehearse,
                      "r_from_broadcast_image": bool(pg)}
    args.r_meta = meta if pg else None
    if args.boundary in ("host", "libsvm", "partition"):
        {"host": bench_host, "libsvm": bench_libsvm, "partition": bench_partition}[args.boundary](
            args, cfg, P, R_host, Ap, Aj, Ax, world, rank, dev)
        if pg:
            dist.destroy_process_group()
        return

    # ---- output buffers sized by an exact first run
    stream = torch.cuda.current_stream(dev).cuda_stream
    if args.staging != "auto" or args.stage_shift:
        P.set_staging(args.staging, args.stage_shift)
    if args.pipeline != "auto":
        P.set_option("pipeline", args.pipeline)
    if args.lpr_chunk_rows is not None:
        P.set_option("chunk_rows", args.lpr_chunk_rows)
    for kv in args.option:
        name, val = kv.split("=", 1)
        P.set_option(name, int(val))
    try:  # full workspace (deferred tile output + staging); the minimal one if HBM is short
        ws = torch.empty(P.workspace_bytes(args.rows, nnz_a, dtype=Ax.dtype), dtype=torch.uint8, device=dev)
    except torch.OutOfMemoryError:
        log(f"[rank {rank}] full workspace does not fit: blocking look-back only")
        ws = torch.empty(P.workspace_bytes(args.rows), dtype=torch.uint8, device=dev)
    cap = int(1.05 * nnz_a * P.nnz / P.m) + 65536
    Cj = torch.empty(cap, dtype=torch.int32, device=dev)
    Cx = torch.empty(cap, dtype=torch.float32, device=dev)
    ip_dtype = torch.int32 if cap < 2**31 else torch.int64
    Cp = torch.empty(args.rows + 1, dtype=ip_dtype, device=dev)
    try:
        nnz_c = P.project_device(Ap, Aj, Ax, Cp, Cj, Cx, order=args.order, stream=stream, workspace=ws, nnz_a=nnz_a)
    except nat.RPError as e:
        if e.code != nat.RP_ERR_CAPACITY:
            raise
        nnz_c = e.nnz
        Cj = torch.empty(nnz_c, dtype=torch.int32, device=dev)
        Cx = torch.empty(nnz_c, dtype=torch.float32, device=dev)
        if nnz_c >= 2**31:
            Cp = torch.empty(args.rows + 1, dtype=torch.int64, device=dev)
        nnz_c = P.project_device(Ap, Aj, Ax, Cp, Cj, Cx, order=args.order, stream=stream, workspace=ws, nnz_a=nnz_a)

    plan = P.plan(args.rows, nnz_a)
    log(f"[rank {rank}] pipeline: {plan}")

    def step():
        k = P.project_device(Ap, Aj, Ax, Cp, Cj, Cx, order=args.order, stream=stream, workspace=ws, nnz_a=nnz_a,
                             sync=args.call == "sync")
        if k is not None and k != nnz_c:
            raise RuntimeError(f"step nnz {k} != first run's {nnz_c}")

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if pg:
        dist.barrier()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(torch.cuda.current_stream(dev))
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    e1.record(torch.cuda.current_stream(dev))
    torch.cuda.synchronize()
    t_wall = time.perf_counter() - t0
    if pg:
        dist.barrier()
    kernel_ms = e0.elapsed_time(e1) / args.steps
    staged_run = P.choice(args.rows, nnz_a, ws)  # auto mode: what the device chose for these rows
    # workspace header (include/rp.h / rp_spgemm.hip Workspace): tiles taken, deferred tiles
    hdr = ws[:24].cpu().numpy().view(np.uint32)
    n_tiles_run, n_deferred = int(hdr[0]), int(hdr[4])
    t_max = _allreduce(t_wall, "max", dev)

    a = nnz_a / args.rows
    c = nnz_c / args.rows
    rbar = P.nnz / P.m
    b_row = algorithmic_bytes_per_row(a, rbar, c)
    achieved = args.rows * b_row / (kernel_ms * 1e-3) / 1e9

    # the timed output, checked after the clock on EVERY rank: a seeded sample of its rows against the
    # oracle (bit for bit), and CSR well-formedness of its whole result on the device; reduced with min
    R_all = _r_host(args, R_host)
    check = verify_output(args, Ap, Aj, Ax, Cp, Cj, Cx, nnz_c, R_all, seed=20261016 + rank)
    ok_all = {k: _allreduce(1.0 if check[k] else 0.0, "min", dev) == 1.0
              for k in ("sample_bitexact_vs_oracle", "indptr_ok", "columns_ok")}
    check = dict(check, **ok_all, ranks_verified=int(_allreduce(1.0 if all(ok_all.values()) else 0.0, "sum", dev)),
                 scope="every rank checks its own rows; flags are the min over ranks")
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:  # host cores, rank 0 only, the other ranks wait
        cpu = cpu_baseline(args, Ap, Aj, Ax, R_all)
    _barrier(dev)
    # boundary 2 beside the headline: the same rows streamed host CSR -> host CSR (PCIe-inclusive);
    # `value` stays the device-resident rate
    boundaries = None
    if args.host_steps > 0:
        h = host_stream_leg(args, P, R_all, Ap, Aj, Ax, world, rank, dev, args.host_steps, 1)
        boundaries = {"host": {
            "rows_per_s": args.rows * world / h["dt"], "ms_per_pass": h["dt"] * 1e3, "steps": args.host_steps,
            "link_frac": h["h2d"] / h["dt"] / 1e9 / PCIE_PEAK_GBS, "h2d_GBps_per_gpu": h["h2d"] / h["dt"] / 1e9,
            "d2h_GBps_per_gpu": h["d2h"] / h["dt"] / 1e9, "host_mem": args.host_mem,
            "stream_stats_rank0": h["stream_stats"],
            "entry": "rp_project_stream (include/rp.h), host CSR in -> host CSR out, PCIe-inclusive",
            "verified": {"sample_rows_per_rank": h["sample_rows"], "sample_bitexact_vs_oracle": bool(h["same"]),
                         "indptr_ok": bool(h["ptr_ok"]), "nnz_out_equal_device_leg": h["nnz_c"] == nnz_c}}}

    # rocprofv3 PMC results of a profiling session of this same workload on THIS build (profiles/):
    # HBM bytes per step and the L2 hit rate of the main kernel. A traffic file applies only when
    # it names the same rows, column distribution, pipeline and librp source hash: a kernel change
    # without a fresh profile reports traffic null, never an old number.
    traffic, traffic_file, tj_used = None, None, {}
    cands = [args.traffic_json] + sorted(glob.glob(os.path.join(ROOT, "profiles", "*traffic*.json")))
    for f in cands:
        try:
            tj = json.load(open(f))
        except Exception:  # noqa: BLE001
            continue
        if (tj.get("rows") == args.rows and tj.get("dist") == args.dist and tj.get("src_sha16") == LIB_ID
                and tj.get("pipeline") == plan["pipeline"] and tj.get("staged") == plan["staged"]
                and tj.get("staged_this_call", staged_run) == staged_run):
            traffic, tj_used = tj.get("hbm_bytes_per_launch"), tj
            traffic_file = os.path.relpath(f, ROOT)
            break
    # L2 behaviour from the same PMC session (null without one for these sources): the hit rate of
    # the kernel that gathers R's descriptors (the staged gather kernel when it ran, else the main
    # kernel), the main kernel's own, and the gathering kernel's measured L2->fabric read requests
    # per second against the ~55 G random lines/s ceiling (scripts/probes/gather_probe*.hip)
    req = tj_used.get("gather_kernel_read_requests_G_per_s")

    if rank == 0:
        total_rows = total_rows_cfg if cfg.get("strong") else args.rows * world
        out = {
            "metric": cfg["metric"],
            "value": total_rows / (t_max / args.steps),
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": t_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if cfg.get("strong") else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": cfg["data"].format(dist=args.dist, p=args.p),
            "config": {"workload": cfg["workload"].format(rows=args.rows, m=args.m, p=args.p),
                       "rows_per_gpu": args.rows, "m": args.m, "p": args.p, "nnz_in": nnz_a, "nnz_out": nnz_c,
                       "order": args.order, "r_layout": P.layout, "parallelism": f"row-shard x{world}",
                       "call": args.call, "options": args.option},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel_ms": kernel_ms, "bytes_per_row": b_row,
                         "model": "B_row=(4+8a)+a(8+8r)+(4+8c)", "a": a, "r": rbar, "c": c,
                         "traffic_source": f"rocprofv3 FETCH_SIZE x2 (gfx950) + WRITE_SIZE per step, {traffic_file}",
                         "l2_hit_rate_r_gathers": tj_used.get("l2_hit_rate_r_gathers"),
                         "l2_hit_rate_r_gathers_scope": tj_used.get("l2_hit_rate_r_gathers_scope"),
                         "l2_hit_rate_gather_kernel": tj_used.get("l2_hit_rate_gather_kernel"),
                         "r_gather_kernel": tj_used.get("gather_kernel"),
                         "l2_hit_rate_main_kernel": tj_used.get("l2_hit_rate_main_kernel"),
                         "pipeline": plan, "librp_src_sha16": LIB_ID,
                         "step_kernels": step_kernels(plan, staged_run, args.call),
                         "traffic_GBps": (traffic / (kernel_ms * 1e-3) / 1e9) if traffic else None,
                         "random_line_ceiling_G_per_s": RANDOM_LINE_CEILING / 1e9,
                         "r_gather_kernel_line_requests_G_per_s": req,
                         "r_gather_kernel_frac_of_random_line_ceiling":
                             (req * 1e9 / RANDOM_LINE_CEILING) if req else None},
            "cpu_baseline": cpu,
            "verified": check,
            "boundaries": boundaries,
            "librp": {"build_id": LIB_ID, "checked_against_sources": LIB_CHECKED, "path": nat.loaded_path()},
            **args.dist_info,
            "r_setup_s": t_r,
            "tiles": n_tiles_run, "deferred_tiles": n_deferred, "staged_this_call": staged_run,
        }
        print(json.dumps(out), flush=True)
    if pg:
        dist.destroy_process_group()


class HostArrays:
    """Host arrays in pageable numpy memory or page-locked memory (rp_host_alloc)."""

    def __init__(self, pinned):
        self.pinned, self.keep = pinned, []

    def empty(self, n, dtype):
        import ctypes

        from randomprojection_amd import _native as nat

        dtype = np.dtype(dtype)
        if not self.pinned:
            a = np.empty(n, dtype)
            a.fill(0)  # fault the pages in (first-touch faults are not part of the measured path)
            return a
        lib = nat.load()
        p = ctypes.c_void_p()
        nat.check(lib.rp_host_alloc(int(n * dtype.itemsize), ctypes.byref(p)))
        self.keep.append(p)
        buf = (ctypes.c_char * int(n * dtype.itemsize)).from_address(p.value)
        return np.frombuffer(buf, dtype=dtype, count=n)

    def free(self):
        from randomprojection_amd import _native as nat

        for p in self.keep:
            nat.load().rp_host_free(p)
        self.keep = []


def _allreduce(x: float, op: str, dev) -> float:
    """max/min/sum of one float over the ranks (gloo rehearsals reduce on the CPU)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return x
    on = dev if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=on)
    dist.all_reduce(t, op={"max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN, "sum": dist.ReduceOp.SUM}[op])
    return float(t.item())


def _barrier(dev):
    import torch
    import torch.distributed as dist

    torch.cuda.synchronize(dev)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


def _r_host(args, R_host):
    """R as host CSR on every rank for the oracle check after the clock: rank 0 built it; the other
    ranks received only the packed device image, so rank 0 broadcasts the CSR arrays once more
    (after the timed region; over RCCL on the device, gloo rehearsals on the CPU)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return R_host
    import scipy.sparse as sp

    meta = args.r_meta
    on = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"
    m, p, nnz = int(meta["m"]), int(meta["p"]), int(meta["nnz"])
    if R_host is not None:
        ts = [torch.from_numpy(np.ascontiguousarray(R_host.indptr, dtype=np.int64)).to(on),
              torch.from_numpy(np.ascontiguousarray(R_host.indices, dtype=np.int32)).to(on),
              torch.from_numpy(np.ascontiguousarray(R_host.data, dtype=np.float32)).to(on)]
    else:
        ts = [torch.empty(m + 1, dtype=torch.int64, device=on), torch.empty(nnz, dtype=torch.int32, device=on),
              torch.empty(nnz, dtype=torch.float32, device=on)]
    for t in ts:
        dist.broadcast(t, src=0)
    if R_host is not None:
        return R_host
    ip, ij, ix = (t.cpu().numpy() for t in ts)
    return sp.csr_matrix((ix, ij, ip), shape=(m, p))


def host_stream_leg(args, P, R_host, Ap, Aj, Ax, world, rank, dev, steps, warmup):
    """Boundary 2: host CSR in -> host CSR out, PCIe-inclusive, through
    rp_project_stream (chunk k+1 uploading while chunk k projects and chunk k-1 downloads). The
    timed region starts with A in host memory and ends with C in host memory. At N ranks every rank
    streams its OWN shard (the recipe's executors, code/clustermode/randomProjection.py:107-113)
    from host memory on its GPU's NUMA node; no collective runs in the loop: a barrier brackets the
    timed steps and the wall time is the max over ranks. Returns the rank-reduced numbers."""
    import torch

    from randomprojection_amd import hostmem

    numa = hostmem.bind_to_device_numa(P.device)  # before the host buffers are allocated and touched
    hm = HostArrays(args.host_mem == "pinned")
    n, nnz_a = args.rows, int(Aj.numel())
    ap = hm.empty(n + 1, np.int32 if nnz_a < 2**31 else np.int64)
    aj, ax = hm.empty(nnz_a, np.int32), hm.empty(nnz_a, np.float32)
    torch.from_numpy(ap).copy_(Ap.to(torch.int64).to(torch.from_numpy(ap).dtype))
    torch.from_numpy(aj).copy_(Aj)
    torch.from_numpy(ax).copy_(Ax)
    exp = nnz_a * P.nnz / P.m
    # host memory is plentiful: room for 25% more than R's mean row length predicts (power-law columns
    # give ~4% more), so the timed passes never take the capacity retry (a second full pass plus a
    # fresh allocation, which the round-5 power-law line measured as its host rate)
    cap = int(1.25 * exp + 8 * np.sqrt(exp)) + 65536
    out = (hm.empty(n + 1, np.int32 if cap < 2**31 else np.int64), hm.empty(cap, np.int32), hm.empty(cap, np.float32))
    order = args.order

    def step():
        r = P.project_stream(ap, aj, ax, order=order, chunk_rows=args.chunk_rows, out=out)
        if r[0] is not out[0]:
            raise RuntimeError("host leg: the output did not fit the caller's arrays (capacity retry)")
        return r

    for _ in range(max(warmup, 1)):
        cp, cj, cx = step()
    _barrier(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        cp, cj, cx = step()
    t_wall = time.perf_counter() - t0
    _barrier(dev)
    dt = _allreduce(t_wall, "max", dev) / steps
    nnz_c = int(cj.size)
    h2d = ap.nbytes + aj.nbytes + ax.nbytes
    d2h = cp.nbytes + cj.nbytes + cx.nbytes
    # after the clock: a seeded sample of this rank's rows against the oracle, bit for bit
    import scipy.sparse as sp

    from oracle import smmp

    rng = np.random.default_rng(20261016 + rank)
    rows = np.sort(rng.choice(n, size=min(4096, n), replace=False))
    A = sp.csr_matrix((ax, aj, ap), shape=(n, args.m))[rows]
    Wp, Wj, Wx, _, _ = smmp.matmat(A, _r_host(args, R_host))
    if order == "sorted":
        Wj, Wx = smmp.sorted_rows(Wp, Wj, Wx)
    C = sp.csr_matrix((cx, cj, cp), shape=(n, args.p))[rows]
    same = (np.array_equal(C.indptr, Wp) and np.array_equal(C.indices, Wj)
            and np.array_equal(C.data.view(np.uint32), Wx.view(np.uint32)))
    res = {
        "dt": dt, "n": n, "nnz_a": nnz_a, "nnz_c": nnz_c, "h2d": h2d, "d2h": d2h, "numa": numa,
        "sample_rows": int(rows.size),
        "same": _allreduce(1.0 if same else 0.0, "min", dev) == 1.0,
        "ptr_ok": _allreduce(1.0 if (cp[0] == 0 and int(cp[-1]) == nnz_c) else 0.0, "min", dev) == 1.0,
        "nnz_max": int(_allreduce(float(nnz_c), "max", dev)),
        "stream_stats": P.stream_stats(),  # this rank's last timed pass (rp_project_stream_stats)
    }
    del A, C, cp, cj, cx, out, ap, aj, ax
    hm.free()
    return res


def bench_host(args, cfg, P, R_host, Ap, Aj, Ax, world=1, rank=0, dev=None):
    """--boundary host: the boundary-2 line on its own (host_stream_leg, args.steps timed passes)."""
    h = host_stream_leg(args, P, R_host, Ap, Aj, Ax, world, rank, dev, args.steps, args.warmup)
    dt, n, h2d, d2h = h["dt"], h["n"], h["h2d"], h["d2h"]
    if rank == 0:
        out_line = {
            "metric": "rows/sec projected (whole node), host CSR in -> host CSR out (PCIe-inclusive, chunked row "
                      "streaming), KDD2012 54.7M->4096 dims",
            "value": n * world / dt, "unit": "rows/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": dt * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32", "data": cfg["data"].format(dist=args.dist, p=args.p),
            "config": {"workload": "configs[1] host boundary: " + cfg["workload"].format(rows=n, m=args.m, p=args.p)
                                   .replace("device-resident CSR in/out", "host CSR in/out"),
                       "boundary": "host", "host_mem": args.host_mem, "chunk_rows": args.chunk_rows or 2 << 20,
                       "rows_per_gpu": n, "nnz_in": h["nnz_a"], "nnz_out": h["nnz_c"],
                       "max_nnz_out_over_ranks": h["nnz_max"], "order": args.order,
                       "parallelism": f"row-shard x{world}, own shard per rank, no collective in the loop",
                       "numa_rank0": h["numa"]},
            "pcie": {"h2d_bytes_per_gpu": h2d, "d2h_bytes_per_gpu": d2h, "h2d_GBps_per_gpu": h2d / dt / 1e9,
                     "d2h_GBps_per_gpu": d2h / dt / 1e9, "host_dram_GBps_node": (h2d + d2h) * world / dt / 1e9,
                     "link_peak_GBps_per_direction": PCIE_PEAK_GBS, "measured_copy_GBps": "H2D ~55, D2H 48-55 "
                     "concurrently (scripts/probes/pcie_probe2.hip)"},
            "roofline": {"bound": "pcie", "achieved": h2d / dt / 1e9, "peak": PCIE_PEAK_GBS, "unit": "GB/s",
                         "frac": h2d / dt / 1e9 / PCIE_PEAK_GBS, "traffic": None,
                         "note": "per GPU: the upload direction binds (92 B/row in vs 53 B/row out); kernel "
                                 "roofline: the device-resident line"},
            "cpu_baseline": None,
            "verified": {"sample_rows_per_rank": h["sample_rows"], "sample_bitexact_vs_oracle": bool(h["same"]),
                         "indptr_ok": bool(h["ptr_ok"])},
            "librp": {"build_id": LIB_ID, "checked_against_sources": LIB_CHECKED},
            **args.dist_info,
        }
        print(json.dumps(out_line), flush=True)


def bench_libsvm(args, cfg, P, R_host, Ap, Aj, Ax, world=1, rank=0, dev=None):
    """Boundary 3: libsvm text in host memory -> GPU parse -> projection -> host
    CSR, through rp_libsvm_project_stream (chunks of whole lines: chunk k+1 uploading while chunk k
    is parsed and projected and chunk k-1 downloads). Replaces spark.read.format("libsvm") + the
    partition function's product (code/clustermode/randomProjection.py:71-72, :46). The text is
    configs[1]-shaped rows written by rp_synth_libsvm_device (values of 6-17 significant digits),
    copied to page-locked host memory before the clock; the timed region starts with the text in
    host memory and ends with labels + CSR in host memory. At N ranks every rank streams its own
    text; no collective in the loop."""
    import ctypes

    import torch

    from randomprojection_amd import hostmem, libsvm, synth

    numa = hostmem.bind_to_device_numa(P.device)
    n = args.rows
    text_d, off_d = synth.libsvm_text_device(Ap, Aj, seed=11 + rank)
    nbytes = int(text_d.numel())
    hm = HostArrays(args.host_mem == "pinned")
    text = hm.empty(nbytes, np.uint8)
    torch.from_numpy(text).copy_(text_d)
    offs = off_d.cpu().numpy()
    nnz_a = int(Aj.numel())
    del text_d, off_d, Ap, Aj, Ax
    torch.cuda.empty_cache()
    exp = nnz_a * P.nnz / P.m
    # host memory is plentiful: room for 25% more than R's mean row length predicts (power-law columns
    # give ~4% more), so the timed passes never take the capacity retry (a second full pass plus a
    # fresh allocation, which the round-5 power-law line measured as its host rate)
    cap = int(1.25 * exp + 8 * np.sqrt(exp)) + 65536
    it = np.int32 if cap < 2**31 else np.int64
    out = (hm.empty(n, np.float64), hm.empty(n + 1, it), hm.empty(cap, np.int32), hm.empty(cap, np.float32))
    order = args.order

    def step():
        return libsvm.project_text_stream(text, P, order=order, chunk_bytes=args.chunk_bytes, out=out)

    for _ in range(max(args.warmup, 1)):
        lab, cp, cj, cx = step()
    _barrier(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        lab, cp, cj, cx = step()
    t_wall = time.perf_counter() - t0
    _barrier(dev)
    dt = _allreduce(t_wall, "max", dev) / args.steps
    nnz_c = int(cj.size)
    # after the clock: a seeded sample of lines parsed by the oracle (Spark's parseLibSVMRecord
    # restated, oracle/libsvm_ref.py) and projected by the scipy-kernel restatement, bit for bit
    import scipy.sparse as sp

    from oracle import smmp
    from oracle.libsvm_ref import parse_text

    rng = np.random.default_rng(20261017 + rank)
    rows = np.sort(rng.choice(n, size=min(2048, n), replace=False))
    sample = b"".join(text[offs[r]:offs[r + 1]].tobytes() for r in rows)
    l_ref, p_ref, j_ref, v_ref = parse_text(sample, args.m)
    A = sp.csr_matrix((v_ref, j_ref, p_ref), shape=(rows.size, args.m))
    Wp, Wj, Wx, _, _ = smmp.matmat(A, _r_host(args, R_host))
    if order == "sorted":
        Wj, Wx = smmp.sorted_rows(Wp, Wj, Wx)
    C = sp.csr_matrix((cx, cj, cp), shape=(n, args.p))[rows]
    same = (int(lab.size) == n and np.array_equal(lab[rows], l_ref) and np.array_equal(C.indptr, Wp)
            and np.array_equal(C.indices, Wj) and np.array_equal(C.data.view(np.uint32), Wx.view(np.uint32)))
    same_all = _allreduce(1.0 if same else 0.0, "min", dev) == 1.0
    d2h = lab.nbytes + cp.nbytes + cj.nbytes + cx.nbytes
    if rank == 0:
        line = {
            "metric": "rows/sec projected (whole node), libsvm text in host memory -> GPU parse + projection -> "
                      "host CSR (PCIe-inclusive, chunked), KDD2012 54.7M->4096 dims",
            "value": n * world / dt, "unit": "rows/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": dt * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic configs[1]-shaped libsvm text (uniform columns, 1+Poisson(10) items per line, values "
                    "with 6-17 significant digits, labels 0/1; rp_synth_libsvm_device), R = "
                    f"SparseRandomProjection({args.p}, random_state=123)",
            "config": {"workload": f"boundary 3: {n} libsvm lines per GPU x {args.m} -> {args.p}, text in "
                                   f"{args.host_mem} host memory, {args.chunk_bytes >> 20} MB chunks",
                       "boundary": "libsvm", "rows_per_gpu": n, "text_bytes_per_gpu": nbytes,
                       "bytes_per_line": nbytes / n, "nnz_in": nnz_a, "nnz_out": nnz_c, "order": order,
                       "parallelism": f"own text per rank x{world}, no collective in the loop", "numa_rank0": numa},
            "text_GBps_per_gpu": nbytes / dt / 1e9,
            "roofline": {"bound": "pcie", "achieved": (nbytes + d2h) / dt / 1e9, "peak": 2 * 63.0, "unit": "GB/s",
                         "frac": (nbytes + d2h) / dt / 1e9 / 126.0, "traffic": None,
                         "h2d_GBps": nbytes / dt / 1e9, "d2h_GBps": d2h / dt / 1e9,
                         "note": "PCIe Gen5 x16 both directions (63 GB/s each); text up, labels + CSR down"},
            "cpu_baseline": None,
            "verified": {"sample_lines_per_rank": int(rows.size), "sample_bitexact_vs_oracle": bool(same_all),
                         "oracle": "oracle/libsvm_ref.py (Spark parseLibSVMRecord + Java double) + oracle/smmp.c"},
            "librp": {"build_id": LIB_ID, "checked_against_sources": LIB_CHECKED},
            **args.dist_info,
        }
        print(json.dumps(line), flush=True)
    hm.free()


def bench_partition(args, cfg, P, R_host, Ap, Aj, Ax, world=1, rank=0, dev=None):
    """Boundary 0, the reference's own (code/clustermode/randomProjection.py:15-54, SURVEY.md §8(a)
    a1): ``random_project_mappartitions_function(rows, R)`` on one partition of ``--part-rows``
    KDD-shaped rows per rank, given as Row-like dicts with SparseVector features (as Spark's
    mapPartitions hands them over) and R as the recipe passes it (``components_.T`` as CSC f32,
    clustermode:101). One step = one call, its lazy output consumed row by row the way a writer
    consumes it (nothing kept). After the clock: where the time goes (each stage timed alone), the
    recipe restated (oracle/recipe.py) on a sample of the same rows on one core of this host, and
    sampled output rows against the oracle, bit for bit."""
    import collections

    import scipy.sparse as sp

    from oracle import smmp
    from oracle.recipe import recipe_partition
    from randomprojection_amd import partition as part
    from randomprojection_amd.linalg import SparseVector

    n = args.rows
    ap = Ap[: n + 1].to(torch_int64()).cpu().numpy()
    aj = Aj[: int(ap[-1])].cpu().numpy()
    ax = Ax[: int(ap[-1])].cpu().numpy().astype(np.float64)  # libsvm values are doubles
    del Ap, Aj, Ax
    m, p = P.m, P.p
    R_all = _r_host(args, R_host)
    R_csc = sp.csc_matrix(R_all)  # local_rnd_mat = srp.components_.T.astype(np.float32): CSC m x p
    t0 = time.perf_counter()
    rows = [{"id": (rank << 40) + i, "label": float(i & 1),
             "features": SparseVector._trusted(m, aj[ap[i]:ap[i + 1]], ax[ap[i]:ap[i + 1]])} for i in range(n)]
    log(f"[rank {rank}] partition of {n} Row dicts built ({time.perf_counter() - t0:.1f}s)")

    def step():
        collections.deque(part.random_project_mappartitions_function(iter(rows), R_csc), maxlen=0)

    for _ in range(max(args.warmup, 1)):  # the first call uploads R (once per R object)
        step()
    _barrier(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t_wall = time.perf_counter() - t0
    _barrier(dev)
    dt = _allreduce(t_wall, "max", dev) / args.steps
    # where the time goes: each stage of the drop-in alone, same partition
    proj = part.get_projector(R_csc)
    t = time.perf_counter()
    ids, labels, has_label, indptr, indices, values, _ = part.assemble_rows(iter(rows))
    t_asm = time.perf_counter() - t
    t = time.perf_counter()
    Cp, Cj, Cx = proj.project_arrays(indptr, indices, values, order="sorted", out_index_dtype=np.int64)
    t_gpu = time.perf_counter() - t
    t = time.perf_counter()
    out = part.random_project_mappartitions_function(iter(rows), R_csc)
    t_call = time.perf_counter() - t  # assemble + GPU + conversions: the call returns the lazy zip
    t = time.perf_counter()
    collections.deque(out, maxlen=0)
    t_mat = time.perf_counter() - t
    # the recipe restated on a sample of the same rows, one core (the reference runs one Python
    # worker per core); R's CSC -> CSR conversion inside its dot is per partition: timed alone
    ns = min(args.recipe_sample_rows, n)
    t = time.perf_counter()
    ref_out = recipe_partition(rows[:ns], R_csc)
    t_rec = time.perf_counter() - t
    t = time.perf_counter()
    sp.csr_matrix(R_csc)
    t_conv = time.perf_counter() - t
    rec_us_row = (t_rec - t_conv) / ns * 1e6 + t_conv / n * 1e6
    # sampled rows of the drop-in's output against the oracle (scipy's kernel restated + sort),
    # and the recipe's own output on its sample
    got = list(part.random_project_mappartitions_function(iter(rows), R_csc))
    rng = np.random.default_rng(20261018 + rank)
    sel = np.sort(rng.choice(n, size=min(2048, n), replace=False))
    A = sp.csr_matrix((ax.astype(np.float32), aj, ap), shape=(n, m))[sel]
    Wp, Wj, Wx, _, _ = smmp.matmat(A, R_all)
    Wj, Wx = smmp.sorted_rows(Wp, Wj, Wx)
    same = len(got) == n
    for k, r in enumerate(sel.tolist()):
        i_, l_, v_ = got[r]
        a, b = Wp[k], Wp[k + 1]
        same &= (i_ == rows[r]["id"] and l_ == rows[r]["label"] and v_.size == p
                 and np.array_equal(v_.indices, Wj[a:b].astype(np.int32))
                 and np.array_equal(v_.values, Wx[a:b].astype(np.float64)))
    same_rec = all(np.array_equal(g[2].indices, q[2].indices) and np.array_equal(g[2].values, q[2].values)
                   and g[0] == q[0] and g[1] == q[1] for g, q in zip(got[:ns], ref_out))
    same_all = _allreduce(1.0 if same and same_rec else 0.0, "min", dev) == 1.0
    del got, ref_out
    if rank == 0:
        line = {
            "metric": "rows/sec projected (whole node), drop-in random_project_mappartitions_function: Row dicts "
                      "in -> (id, label, SparseVector) tuples out, KDD2012 54.7M->4096 dims",
            "value": n * world / dt, "unit": "rows/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": dt * 1e3, "us_per_row": dt / n * 1e6, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": cfg["data"].format(dist=args.dist, p=args.p),
            "config": {"workload": f"boundary 0: one partition of {n} KDD2012-shaped Row dicts per rank (one "
                                   "Python process per GPU), R = components_.T CSC f32 as the recipe passes it",
                       "boundary": "partition", "part_rows": n, "parallelism": f"one partition per rank x{world}"},
            "where_time_goes_ms": {"assemble_rows": t_asm * 1e3, "gpu_project_host_arrays": t_gpu * 1e3,
                                   "call_returns_lazy_zip": t_call * 1e3,
                                   "output_rows_materialised_streamed": t_mat * 1e3},
            "cpu_baseline": {"value": 1e6 / rec_us_row, "unit": "rows/s", "cores": 1, "kind": "port",
                             "us_per_row": rec_us_row,
                             "sample": f"the recipe restated (oracle/recipe.py = clustermode:15-54 step for step), "
                                       f"first {ns} rows of the same partition on one core; its per-call R CSC->CSR "
                                       f"conversion ({t_conv:.2f} s) charged once per {n}-row partition",
                             "sample_s": t_rec, "r_conversion_s": t_conv},
            "speedup_vs_recipe_per_process": rec_us_row / (dt / n * 1e6),
            "verified": {"sample_rows_per_rank": int(sel.size), "sample_bitexact_vs_oracle": bool(same_all),
                         "recipe_sample_equal": "included in the flag (first sample rows vs oracle/recipe.py)"},
            "librp": {"build_id": LIB_ID, "checked_against_sources": LIB_CHECKED},
            **args.dist_info,
        }
        print(json.dumps(line), flush=True)


def torch_int64():
    import torch

    return torch.int64


def verify_output(args, Ap, Aj, Ax, Cp, Cj, Cx, nnz_c, R_host, n_sample=4096, seed=20261016):
    """After the timed region: Cp monotone from 0 to nnz, every column in [0, p), and a seeded
    sample of rows (spread over the whole matrix) equal to the oracle's restatement of scipy's
    csr_matmat, bit for bit (indices in scipy's per-row order, or ascending for --order sorted, and
    value bits)."""
    import scipy.sparse as sp
    import torch

    from oracle import smmp

    cp = Cp.to(torch.int64)
    ok_ptr = bool(cp[0].item() == 0 and cp[-1].item() == nnz_c and torch.all(cp[1:] >= cp[:-1]).item())
    cj = Cj[:nnz_c]
    ok_cols = bool(nnz_c == 0 or (int(cj.min().item()) >= 0 and int(cj.max().item()) < args.p))
    rng = np.random.default_rng(seed)
    rows = np.sort(rng.choice(args.rows, size=min(n_sample, args.rows), replace=False))
    r_t = torch.as_tensor(rows, device=Ap.device)
    s0, s1 = Ap[r_t].to(torch.int64).cpu().numpy(), Ap[r_t + 1].to(torch.int64).cpu().numpy()
    c0, c1 = cp[r_t].cpu().numpy(), cp[r_t + 1].cpu().numpy()

    def take(t, lo, hi):  # the sampled rows' segments of a device array, gathered on the device
        idx = np.concatenate([np.arange(a, b) for a, b in zip(lo, hi)]).astype(np.int64)
        return t[torch.as_tensor(idx, device=t.device)].cpu().numpy()

    ptr = np.concatenate([[0], np.cumsum(s1 - s0)])
    A = sp.csr_matrix((take(Ax, s0, s1), take(Aj, s0, s1), ptr), shape=(rows.size, args.m))
    Wp, Wj, Wx, _, _ = smmp.matmat(A, R_host)
    if args.order == "sorted":
        Wj, Wx = smmp.sorted_rows(Wp, Wj, Wx)
    got_ptr = np.concatenate([[0], np.cumsum(c1 - c0)])
    same = (np.array_equal(got_ptr, Wp) and np.array_equal(take(Cj, c0, c1), Wj)
            and np.array_equal(take(Cx, c0, c1).view(np.uint32), Wx.view(np.uint32)))
    return {"sample_rows": int(rows.size), "sample_bitexact_vs_oracle": bool(same),
            "indptr_ok": ok_ptr, "columns_ok": ok_cols}


def cpu_baseline(args, Ap, Aj, Ax, R_host):
    """the reference's CPU path timed on this box's host cores, on a bounded sample
    of the same workload, in a child process (oracle/cpu_baseline.py; this process holds the GPU,
    the child forks one worker per core): (i) the recipe restated (oracle/recipe.py), one process
    per core on partitions of part_rows rows -> `value`; (ii) scipy's kernel pair restated
    (oracle/smmp.c) on N threads; each with a 1-core figure. kind "port": restatements (the
    reference's own Python cannot travel to the box)."""
    import subprocess
    import tempfile

    part = args.cpu_part_rows
    krows = min(args.cpu_sample_rows, args.rows)
    n = max(krows, part * 64)
    n = min(n, args.rows)
    ap = Ap[: n + 1].cpu().numpy().astype(np.int64)
    e = int(ap[-1])
    base = "/dev/shm" if os.access("/dev/shm", os.W_OK) else None
    with tempfile.TemporaryDirectory(dir=base, prefix="rp_cpu_") as d:
        np.save(os.path.join(d, "ap.npy"), (ap - ap[0]).astype(np.int64))
        np.save(os.path.join(d, "aj.npy"), Aj[int(ap[0]):e].cpu().numpy())
        np.save(os.path.join(d, "ax.npy"), Ax[int(ap[0]):e].cpu().numpy())
        np.save(os.path.join(d, "rp.npy"), R_host.indptr.astype(np.int32))
        np.save(os.path.join(d, "rj.npy"), R_host.indices.astype(np.int32))
        np.save(os.path.join(d, "rx.npy"), R_host.data.astype(np.float32))
        np.save(os.path.join(d, "p.npy"), np.int64(R_host.shape[1]))
        env = dict(os.environ, PYTHONPATH=ROOT)
        r = subprocess.run([sys.executable, "-m", "oracle.cpu_baseline", d, str(R_host.shape[0]), str(part),
                            str(krows)], cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        log(r.stderr[-2000:])
        raise RuntimeError(f"cpu baseline child failed ({r.returncode})")
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    rec, ker = res["recipe"], res["kernel_port"]
    return {"value": rec["value"], "unit": "rows/s", "cores": res["cores"], "kind": "port",
            "sample": f"(i) the recipe restated (oracle/recipe.py: per-row COO->CSR, vstack, CSR @ CSC R, sorted "
                      f"per-row SparseVector output), {rec['processes']} processes x {rec['part_rows']} rows of the "
                      f"same synthetic workload, one partition each, started together",
            "one_core": rec["one_core"],
            "affinity_cpus": res["affinity_cpus"], "cgroup_quota_cpus": res["cgroup_quota_cpus"],
            "recipe": rec,
            "kernel_port": dict(ker, unit="rows/s",
                                note="(ii) scipy csr_matmat_maxnnz + csr_matmat restated (oracle/smmp.c), first "
                                     f"{ker['rows']} rows, {ker['threads']} threads")}


if __name__ == "__main__":
    main()

"""Benchmark: MicroRank RCA windows on MI355X (one process per GPU).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--precision fp64|fp32] [--no-cpu]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (driver, N > 1)

Workload (BASELINE.json configs[1], "C2"): RCA windows of 1k operations / 200k traces each
(~13.7 spans per trace, ~2.74M spans per window; Train-Ticket-like synthetic call tree with one
faulty operation), fp64.  The span columns are generated, factorised and uploaded BEFORE the
timed region; a window is ranked on the device: detector -> two graph builds (T1 swap) -> two
25-iteration PageRanks -> DStar2 spectrum + top list.  A "step" ranks DISTINCT windows (own
seed and span table each; 256 per step) with ONE mr_windows_batch call (their detectors / builds / spectra on
the library's auxiliary streams, the PageRanks of a group of windows sharing each iteration's
launches).

N > 1: every rank ranks its own independent windows (different seed): data-parallel windows,
no collective on the data path -> "scaling": "weak".  Beside the headline
the line carries "c4_sharded": ONE C4 graph (10k ops / 10M traces, BASELINE configs[3]) split by
trace over the N ranks (strong scaling: 10M/N traces per rank), a whole trace_pagerank per step
with the per-iteration exact-limb all-reduce (IPC peer push over xGMI, RCCL fallback) -- the
north star's >= 6x-at-8-GPUs workload, so the driver's 1/2/4/8 run yields its curve.

value = edges traversed by all PageRank iterations of all ranks (25 * (2 nnz + E_c) per graph)
/ max-over-ranks wall time of the K steps  [GTEPS].  Every other part of the window (detector,
graph builds, spectrum) is inside that time.  windows_per_s is reported beside it.
roofline: one power iteration (the k_tr_a + k_fx_b launch pair over a window group's graphs),
algorithmic bytes (SURVEY §8(d) B_iter of every graph of the launch) over its live HIP-event
duration on the library's stream; traffic = FETCH_SIZE (x2, gfx950) + WRITE_SIZE of the same
launches per iteration from two rocprofv3 --pmc child runs made before this process touches the
GPU (--no-traffic skips them).  roofline.fracs puts the three fractions side by side: SURVEY
bytes (4-B op ids), the bytes the walk reads (u16 ids), PMC bytes.  The timed walk visits every
trace (no kind compression of any form); the run-merged walk -- SURVEY 8(f)4's compression
inside k_tr_a -- is its own side leg (value_run_merged, roofline.run_merged).  --no-side: the timed steps only (no single-window latency, kind-
compressed probe or c4_sharded leg), so a rocprofv3 kernel table of the command holds only the
timed shape's launches (profiles/README.md).
cpu_baseline: the C restatement (oracle/, OpenMP) of the same window on this host's cores.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s HBM3E spec


def make_window(seed: int, n_ops: int, n_traces: int):
    """Synthetic C2 window: (SpanTable of the window, SpanTable of the normal SLO period)."""
    from microrank_amd import synth

    topo, normal, abnormal = synth.window_pair(n_ops, n_traces, seed, branch=1.9, p_max=0.8, fault_ms=6000.0,
                                               names=False)
    for st in (normal, abnormal):
        st.trace_names = None
    return topo, normal, abnormal


def _c2_abnormal(job):
    """One distinct C2 window's spans (process-pool worker): the shared topology, its own seed."""
    from microrank_amd import synth

    topo, n_traces, seed = job
    st = synth.gen_spans(topo, n_traces, seed, branch=1.9, p_max=0.8, fault_op=synth.fault_op_of(topo),
                         fault_frac=0.4, fault_ms=6000.0, names=False)
    st.trace_names = None
    st.meta = {}
    return st


def c2_windows(n: int, n_ops: int, n_traces: int, rank: int):
    """n DISTINCT C2 windows of one system (BASELINE configs[1]: 1k ops / 200k traces each): one
    topology and normal SLO period, each window's traffic from its own seed (a 5-minute window of a
    different time).  Generated in a process pool before this process touches the GPU.  Returns
    (normal SpanTable, [abnormal SpanTable] * n)."""
    from concurrent.futures import ProcessPoolExecutor

    seed = 1234 + 7919 * rank
    topo, normal, first = make_window(seed, n_ops, n_traces)
    jobs = [(topo, n_traces, seed + 2 + 104729 * i) for i in range(1, n)]
    threads, _ = host_cores()
    if not jobs:
        return normal, [first]
    with ProcessPoolExecutor(max_workers=max(1, min(16, threads, len(jobs)))) as ex:
        rest = list(ex.map(_c2_abnormal, jobs))
    return normal, [first] + rest


def slo_from_gpu(ctx, normal):
    """SLO of the normal period with K4 (get_operation_slo's kernel), as {svcop code: a3}."""
    import ctypes as C

    from microrank_amd import _lib
    from microrank_amd._lib import ptr
    from microrank_amd.preprocess_data import DeviceSpans

    dev = DeviceSpans(ctx, normal)
    n = normal.n_svcops
    mean, std, cnt = np.empty(n), np.empty(n), np.empty(n, np.int64)
    ctx.check(_lib.load().mr_slo(ctx.h, dev.h, ptr(mean, C.c_double), ptr(std, C.c_double), ptr(cnt, C.c_int64)))
    dev.close()
    a3 = mean + 3 * std
    ok = (cnt > 0).astype(np.uint8)
    return a3, ok


def run_window(ctx, dev, t0, t1, a3, ok, prec):
    import ctypes as C

    from microrank_amd import _lib
    from microrank_amd._lib import ptr

    codes = np.zeros(11, np.int32)
    scores = np.zeros(11, np.float64)
    n_out, na, nn, edges = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int64()
    ctx.check(_lib.load().mr_rca_window(ctx.h, dev.h, t0, t1, ptr(a3, C.c_double), ptr(ok, C.c_uint8), 0, 5, prec,
                                        ptr(codes, C.c_int32), ptr(scores, C.c_double), C.byref(n_out),
                                        C.byref(edges), C.byref(na), C.byref(nn)), "mr_rca_window")
    return edges.value, codes[:n_out.value].copy(), scores[:n_out.value].copy(), na.value, nn.value


ITER_KERNELS = ("k_tr_a", "k_fx_b", "k_iter_a", "k_iter_b", "k_cold_trace", "k_cold_ops")


def copy_peak(ctx, nbytes=1 << 30, reps=5):
    """This GPU's measured STREAM-copy rate (the roofline against a measured copy
    peak beside the 8 TB/s spec): mr_copy_peak, a 16-B-per-lane copy of 1 GiB, best of 5."""
    import ctypes as C

    from microrank_amd import _lib

    g = C.c_double()
    ctx.check(_lib.load().mr_copy_peak(ctx.h, int(nbytes), int(reps), C.byref(g)), "mr_copy_peak")
    return g.value


def add_copy_frac(out, ctx):
    """roofline.copy_peak and every roofline fraction also against it (frac_vs_copy)."""
    try:
        cp = copy_peak(ctx)
    except Exception as e:  # a side metric never sinks the line
        out["roofline"]["copy_peak"] = {"error": f"{type(e).__name__}: {e}"}
        return
    r = out["roofline"]
    r["copy_peak"] = round(cp, 1)
    # against the copy peak on the bytes a launch MOVES: SURVEY's B_iter counts 4-B op ids where
    # the walk reads 2-B ones, so its figures are scaled by the u16 / SURVEY byte ratio first (a
    # SURVEY-byte rate above the copy peak is not a rate the kernel ran at)
    mv = 1.0
    if isinstance(r.get("u16_ids"), dict) and r.get("bytes_per_launch"):
        mv = r["u16_ids"]["bytes_per_launch"] / r["bytes_per_launch"]
    wr = out.get("window_roofline") if isinstance(out.get("window_roofline"), dict) else None
    for d, f in [(r, mv)] + [(r[k], mv if k in ("isolated", "run_merged") else 1.0)
                             for k in ("u16_ids", "pmc_bytes", "isolated", "run_merged") if isinstance(r.get(k), dict)] + \
                ([(wr, wr.get("moved_bytes_per_window", 0) / wr["bytes_per_window"])] if wr and wr.get("bytes_per_window") else []):
        if isinstance(d.get("achieved"), (int, float)) and cp > 0 and f > 0:
            d["frac_vs_copy"] = round(d["achieved"] * f / cp, 4)
    r["frac_vs_copy_what"] = "achieved x (bytes moved, 2-B op ids / the figure's bytes) / copy_peak"
    if isinstance(r.get("fracs"), dict) and cp > 0:
        r["fracs"]["copy_peak_frac_of_spec"] = round(cp / HBM_PEAK_GBS, 4)


def add_pmc_frac(out, traffic):
    """roofline.pmc_bytes: the same launches on the HBM bytes the PMC counters saw (traffic per
    iteration over the live per-iteration time), and roofline.fracs: the three fractions side by
    side -- SURVEY 8(d) bytes (4-B op ids), the bytes the walk reads (2-B ids), PMC bytes."""
    r = out["roofline"]
    avg_us = r.get("avg_launch_us") or 0.0
    if traffic is not None and avg_us > 0:
        pb = traffic["fetch"] + traffic["write"]
        r["pmc_bytes"] = {"bytes_per_launch": round(pb), "achieved": round(pb / (avg_us * 1e-6) / 1e9, 1),
                          "frac": round(pb / (avg_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                          "what": "rocprofv3 FETCH_SIZE (x2) + WRITE_SIZE per iteration / the live iteration time"}
    r["fracs"] = {"survey_bytes": r.get("frac"),
                  "u16_bytes": r["u16_ids"]["frac"] if isinstance(r.get("u16_ids"), dict) else None,
                  "pmc_bytes": r["pmc_bytes"]["frac"] if isinstance(r.get("pmc_bytes"), dict) else None}


def kind_compressed_probe(ctx, dev, t0, t1, a3, ok, reps=5):
    """§8(f) f4, reported beside (not in) GTEPS: the window's larger graph (the detector's normal
    traces) ranked uncompressed and kind-compressed (MR_PR_KIND_COMPRESS: one representative per
    trace kind, multiplicities carried): time per trace_pagerank call, kinds vs traces, and the
    largest relative weight difference."""
    import ctypes as C

    from microrank_amd import _lib
    from microrank_amd._lib import ptr
    from microrank_amd.graph import DeviceGraph

    lib = _lib.load()
    n_tr = dev.table.n_traces
    state = np.zeros(n_tr, np.uint8)
    na, nn, nin = C.c_int32(), C.c_int32(), C.c_int64()
    ctx.check(lib.mr_detect(ctx.h, dev.h, t0, t1, ptr(a3, C.c_double), ptr(ok, C.c_uint8), ptr(state, C.c_uint8),
                            C.byref(na), C.byref(nn), C.byref(nin)), "mr_detect")
    mask = (state == 1).astype(np.uint8)
    h = _lib.P()
    ctx.check(lib.mr_graph_build(ctx.h, dev.h, ptr(mask, C.c_uint8), C.byref(h)), "mr_graph_build")
    n, t, nnz, e = C.c_int32(), C.c_int32(), C.c_int64(), C.c_int64()
    lib.mr_graph_info(h, C.byref(n), C.byref(t), C.byref(nnz), C.byref(e))
    g = DeviceGraph(ctx, h, None, None, n.value, t.value)
    res, first = {}, {}
    for comp in (False, True):
        ctx.sync()
        ts = time.perf_counter()
        g.pagerank(True, compress_kinds=comp)   # compressed: builds the representatives' graph
        ctx.sync()
        first[comp] = (time.perf_counter() - ts) * 1e3
        ts = time.perf_counter()
        for _ in range(reps):
            g.pagerank(True, compress_kinds=comp)
        ctx.sync()
        res[comp] = ((time.perf_counter() - ts) / reps * 1e3, *g.fetch(kinds=True)[:3])
    w0, w1, kind = res[False][1], res[True][1], res[True][3]
    g.close()
    return {"graph": f"C2 window, detector-normal traces: {t.value} traces / {n.value} ops / {nnz.value} pairs",
            "kinds": int(round(float((1.0 / kind).sum()))), "traces": int(t.value),
            "ms_per_call": round(res[True][0], 3), "ms_per_call_uncompressed": round(res[False][0], 3),
            "speedup": round(res[False][0] / res[True][0], 3),
            "ms_first_call": round(first[True], 3),
            "what": "ms_per_call: later calls on the graph (its representatives' graph kept, per-call "
                    "preference + 25 iterations + weights); ms_first_call: the call that builds it",
            "max_rel_diff": float(np.max(np.abs(w1 - w0) / np.maximum(np.abs(w0), 1e-300)))}


def pmc_traffic(args, timeout_s=240):
    """HBM bytes per power iteration (all kernels of one iteration: k_tr_a + k_fx_b, or the tile
    path's k_iter_a + k_iter_b) from two rocprofv3 --pmc child runs of this bench (FETCH_SIZE and
    WRITE_SIZE in separate passes, MI355X_MICROARCH.md 'HBM': FETCH_SIZE reads half the bytes of
    wide streaming loads on gfx950 -> x2).  Child processes only: this process has not touched
    the GPU yet when it runs them.  None when rocprofv3 is unavailable or a pass fails."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile

    prof = shutil.which("rocprofv3") or ("/opt/rocm/bin/rocprofv3" if os.path.exists("/opt/rocm/bin/rocprofv3") else None)
    if prof is None:
        return None
    env = dict(os.environ, TMPDIR="/tmp")
    vals = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        with tempfile.TemporaryDirectory(dir="/tmp") as d:
            cmd = [prof, "--pmc", ctr, "-d", d, "-o", "run", "--output-format", "csv", "--",
                   sys.executable, os.path.abspath(__file__), "--pmc-child", "--steps", "2", "--warmup", "1",
                   "--no-cpu", "--precision", args.precision]
            if args.config in ("c4", "c5"):
                cmd += ["--config", args.config, "--c4-ops", str(args.c4_ops), "--c4-traces", str(args.c4_traces)]
            else:
                cmd += ["--streams", str(args.streams), "--ops", str(args.ops), "--traces", str(args.traces)]
                if args.config == "c2":   # (the same launches; 64 distinct windows cycled: less generation)
                    cmd += ["--c2-distinct", "64"]
            try:
                subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                               timeout=timeout_s, check=True)
            except Exception:
                return None
            per_iter, n_a = 0.0, 0
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                for r in csv.DictReader(open(f)):
                    name = r["Kernel_Name"]
                    if r["Counter_Name"] == ctr and any(k in name for k in ITER_KERNELS):
                        per_iter += float(r["Counter_Value"])
                        n_a += any(k in name for k in ("k_tr_a", "k_iter_a"))   # one walk launch per iteration
            if n_a == 0:
                return None
            vals[ctr] = per_iter / n_a * 1024.0   # KB -> bytes, per iteration
    return {"fetch": 2.0 * vals["FETCH_SIZE"], "write": vals["WRITE_SIZE"]}


def host_cores():
    """(threads this process may use, CPUs of the machine): the CPU affinity / OMP_NUM_THREADS share
    (16 per GPU on the GPU box, whose nproc shows the whole machine) and os.cpu_count()."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return (min(aff, omp) if omp > 0 else aff), (os.cpu_count() or 1)


def cpu_baseline(abnormal, t0, t1, a3, ok, target_s=10.0, one_core_s=8.0):
    """The oracle's C restatement of the same window, timed on this host (bounded samples): on
    every core this process may use, and on one core (SURVEY §8(d) CPU baseline timing)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import c_oracle

    threads, machine = host_cores()
    res = c_oracle.rca_window(abnormal, t0, t1, a3, ok, nthreads=threads)   # warm-up + correctness handle

    def timed(nthreads, budget, cap):
        n, t_start, edges = 0, time.perf_counter(), 0
        while True:
            r = c_oracle.rca_window(abnormal, t0, t1, a3, ok, nthreads=nthreads)
            edges += r[4]
            n += 1
            el = time.perf_counter() - t_start
            if el >= budget or n >= cap:
                return n, el, edges

    n, el, edges = timed(threads, target_s, 20)
    n1, el1, edges1 = timed(1, one_core_s, 8)
    return {"value": round(edges / el / 1e9, 4), "unit": "GTEPS", "cores": threads, "kind": "port",
            "sample": f"{n} full windows of this config (detect + 2 graph builds + 2x25 PageRank iterations + spectrum), "
                      f"oracle/mr_oracle.c OpenMP on {threads} threads, {el:.1f} s; one core: {n1} windows, {el1:.1f} s",
            "windows_per_s": round(n / el, 4), "nproc": machine,
            "one_core": {"value": round(edges1 / el1 / 1e9, 4), "windows_per_s": round(n1 / el1, 4), "cores": 1}}, res


def c4_cpu_baseline(hg, anomaly=True, one_core_iters=2):
    """SURVEY 8(d) CPU baseline of a C4 / C5 step on the same graph the GPU ranks: the C restatement
    (oracle/mr_oracle.c oracle_incidence_pagerank: kinds by column hash + exact check, preference,
    25 OpenMP power iterations, weights) on every core this process may use, one whole
    trace_pagerank; on one core, kinds + preference and `one_core_iters` iterations, the 25-iteration
    time extrapolated from them (a bounded sample).  GTEPS = 25 (2 nnz + E) / time, as the GPU line."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import c_oracle

    threads, machine = host_cores()
    edges = 25.0 * (2.0 * float(hg.sr_ops.size) + float(hg.ss_par.size))
    ts = time.perf_counter()
    _, _, tp = c_oracle.incidence_pagerank(hg, anomaly, 25, nthreads=threads)
    t_all = tp[0] + tp[1]
    el = time.perf_counter() - ts
    _, _, tp1 = c_oracle.incidence_pagerank(hg, anomaly, one_core_iters, nthreads=1)
    t_one = tp1[0] + tp1[1] * 25.0 / one_core_iters
    return {"value": round(edges / t_all / 1e9, 4), "unit": "GTEPS", "cores": threads, "kind": "port",
            "sample": f"one whole trace_pagerank of this graph ({hg.T} traces / {hg.N} ops: kinds + preference "
                      f"{tp[0]:.2f} s, 25 iterations + weights {tp[1]:.2f} s) by oracle/mr_oracle.c on {threads} "
                      f"OpenMP threads ({el:.1f} s wall incl. the op-major copy); one core: kinds + preference "
                      f"{tp1[0]:.2f} s + {one_core_iters} iterations {tp1[1]:.2f} s, extrapolated to 25",
            "ms_per_step": round(t_all * 1e3, 1), "nproc": machine,
            "one_core": {"value": round(edges / t_one / 1e9, 4), "cores": 1, "ms_per_step_est": round(t_one * 1e3, 1)}}


def run_c4(args, world, rank, dist):
    """C4: one 10k-op / 10M-trace graph sharded by trace over the ranks (strong scaling); a step is
    one whole trace_pagerank of the graph (kinds, preference, 25 iterations with the per-iteration
    exact limb all-reduce over RCCL)."""
    import ctypes as C

    from microrank_amd import _lib, shard, synth
    from microrank_amd.graph import DeviceGraph

    # --shard-of K at N = 1: this GPU holds rank 0's share of a K-rank deployment
    sw, sr = (world, rank) if world > 1 else (max(1, args.shard_of), 0)
    t_local = args.c4_traces // sw + (1 if sr < args.c4_traces % sw else 0)
    t_gen = time.perf_counter()
    ctx = _lib.default_context()
    if world > 1:
        shard.use_rccl(ctx)   # the once-per-graph collectives (and the fallback per iteration)
        if not os.environ.get("MR_BENCH_NO_PEER"):
            shard.use_peer(ctx)   # per iteration: IPC peer push over xGMI (falls back to RCCL collectively)
    prec = args.precision
    # N <= FX_NMAX: k_tr_a + k_fx_b; above it the wide fused path (hot ops through k_tr_a, cold
    # entries through k_cold_trace / k_cold_ops); MR_NO_WIDE=1 keeps the tile path for A/B runs
    wide = args.c4_ops > 16384
    fused = not (wide and os.environ.get("MR_NO_WIDE"))
    dev = None
    if args.from_spans:
        # K1 inside the timed step: this rank's span shard is resident in HBM (ingest), a step
        # builds the rank's graph from it (mr_graph_build_sharded: global node order and
        # cross-rank parent joins over the collectives) and ranks it
        from microrank_amd.preprocess_data import DeviceSpans

        st = synth.big_spans(args.c4_ops, args.c4_traces, seed=11, shard=(sr, sw))
        print(f"[bench] rank {rank}: generated {t_local} traces / {st.n_spans} spans in "
              f"{time.perf_counter() - t_gen:.1f} s", file=sys.stderr, flush=True)
        dev = DeviceSpans(ctx, st)
        mask = np.ones(st.n_traces, np.uint8)
        n_spans_local = st.n_spans
        del st
        dg = None
    else:
        hg = synth.big_graph(args.c4_ops, t_local, seed=11, shard=(rank, world))
        print(f"[bench] rank {rank}: generated {t_local} traces / {hg.sr_ops.size} pairs in "
              f"{time.perf_counter() - t_gen:.1f} s", file=sys.stderr, flush=True)
        dg = DeviceGraph.upload(ctx, hg)
        if world > 1 or args.no_cpu:
            del hg   # (kept on rank 0 at N = 1: the CPU baseline ranks the same graph)
    build_s = [0.0]

    def step():
        nonlocal dg
        if dev is not None:
            if dg is not None:
                dg.close()
            tb = time.perf_counter()
            dg = shard.build_graph(dev, mask)
            ctx.sync()
            build_s[0] += time.perf_counter() - tb
        return shard.sharded_pagerank(dg, True, precision=prec)

    for _ in range(max(args.warmup, 1)):   # the first call also runs the once-per-graph exchange
        step()
    E = dg.info()["E"]
    nnz_local = dg.info()["nnz"]
    load = _lib.load()
    load.mr_ctx_profile(ctx.h, 1)
    ctx.sync()
    if dist is not None:
        dist.barrier()
    build_s[0] = 0.0
    t_start = time.perf_counter()
    for _ in range(args.steps):
        w, cov = step()
    ctx.sync()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    launches, kms, kbytes = C.c_int64(), C.c_double(), C.c_double()
    load.mr_ctx_prof_read(ctx.h, C.byref(launches), C.byref(kms), C.byref(kbytes))
    nnz_all = float(nnz_local)
    if dist is not None:
        import torch

        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t[0])
        t = torch.tensor([nnz_all], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        nnz_all = float(t[0])
    if rank != 0:
        return None
    avg_ms = kms.value / max(launches.value, 1)
    achieved = (kbytes.value / max(launches.value, 1)) / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    edges = 25.0 * (2.0 * nnz_all + E) * args.steps
    out = {
        "metric": "PageRank GTEPS + RCA windows ranked/sec at 1/2/4/8 MI355X; % HBM roofline",
        "value": round(edges / elapsed / 1e9, 3), "unit": "GTEPS", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64" if prec == "fp64" else "f32",
        "data": "synthetic (power-law op popularity, root op in every trace, random call tree; per-rank shards)",
        "config": {"workload": f"{args.config.upper()} sharded "
                               + ("K1 graph build from span shards + " if dev is not None else "")
                               + f"trace_pagerank: {args.c4_ops} ops / {args.c4_traces} "
                               f"traces over {world} GPU(s), anomaly preference, 25 iterations"
                               + (f"; this GPU: rank 0's share of {sw} ({t_local} traces)" if sw != world else ""),
                   "nnz": int(nnz_all),
                   "call_edges": E,
                   "parallelism": f"trace shards x{world}, "
                                  + (("IPC peer push" if shard.peer_active(ctx) else "RCCL") if world > 1 else "no")
                                  + (" limb" if fused else " fp64 op-sum") + " all-reduce per iteration"},
        "roofline": {"bound": "hbm", "kernel": "one Jacobi iteration on this rank ("
                                               + (("k_cold_trace + k_cold_ops + k_tr_a + k_fx_b" if wide else
                                                   "k_tr_a + k_fx_b") if fused else "k_iter_a + k_iter_b")
                                               + (" + 2 all-reduces)" if world > 1 else ")"),
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "avg_launch_us": round(avg_ms * 1e3, 3), "launches": launches.value,
                     "bytes_per_launch": round(kbytes.value / max(launches.value, 1))},
    }
    if fused and not wide and avg_ms > 0:   # the same iteration on the bytes it moves: u16 op ids, not SURVEY's 4-B ids
        b16 = kbytes.value / max(launches.value, 1) - 2.0 * float(nnz_local)
        out["roofline"]["u16_ids"] = {"bytes_per_launch": round(b16), "achieved": round(b16 / (avg_ms * 1e-3) / 1e9, 1),
                                      "frac": round(b16 / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    if dev is not None:
        out["data"] = ("synthetic span shards (power-law ops, root op in every trace, random parent per span, "
                       "5% broken traces, 1% duplicated root spanIDs across ranks), int-coded, resident in HBM")
        out["config"]["n_spans_rank0"] = int(n_spans_local)
        out["build_ms"] = round(build_s[0] / args.steps * 1e3, 3)   # rank 0's K1 share of a step
    add_copy_frac(out, ctx)
    if not args.no_cpu and world == 1 and dev is None:
        try:
            out["cpu_baseline"] = c4_cpu_baseline(hg)
        except Exception as e:
            out["cpu_baseline"] = {"value": None, "error": f"{type(e).__name__}: {e}"}
    return out


C4_OPS, C4_TRACES = 10_000, 10_000_000   # BASELINE configs[3]


def c4_leg_generate(world, rank):
    """This rank's share of the C4 graph for the default line's c4_sharded leg (generated before
    the process touches the GPU: the generator forks a process pool)."""
    from microrank_amd import synth

    t_local = C4_TRACES // world + (1 if rank < C4_TRACES % world else 0)
    ts = time.perf_counter()
    hg = synth.big_graph(C4_OPS, t_local, seed=11, shard=(rank, world))
    print(f"[bench] rank {rank}: c4_sharded shard {t_local} traces / {hg.sr_ops.size} pairs in "
          f"{time.perf_counter() - ts:.1f} s", file=sys.stderr, flush=True)
    return hg


def c4_leg_run(hg, world, rank, dist, steps=10, warmup=2):
    """The c4_sharded leg: ONE 10k-op / 10M-trace graph split by trace over the ranks (strong
    scaling), a step = one whole trace_pagerank (kinds, preference, 25 iterations with one exact
    limb all-reduce each: IPC peer push over xGMI, RCCL fallback).  Max-over-ranks wall time.
    The driver's N = 1/2/4/8 runs of the default command give the north star's C4 curve."""
    import ctypes as C

    import torch

    from microrank_amd import _lib, shard
    from microrank_amd.graph import DeviceGraph

    ctx = _lib.Context(int(os.environ.get("MICRORANK_DEVICE", "0")))
    if world > 1:
        shard.use_rccl(ctx)
        if not os.environ.get("MR_BENCH_NO_PEER"):
            shard.use_peer(ctx)
    dg = DeviceGraph.upload(ctx, hg)
    nnz = float(dg.info()["nnz"])
    for _ in range(warmup):
        shard.sharded_pagerank(dg, True)
    E = dg.info()["E"]
    lib = _lib.load()
    lib.mr_ctx_profile(ctx.h, 1)
    ctx.sync()
    if dist is not None:
        dist.barrier()
    ts = time.perf_counter()
    for _ in range(steps):
        w, _cov = shard.sharded_pagerank(dg, True)
    ctx.sync()
    if dist is not None:
        dist.barrier()
    el = time.perf_counter() - ts
    launches, kms, kbytes = C.c_int64(), C.c_double(), C.c_double()
    lib.mr_ctx_prof_read(ctx.h, C.byref(launches), C.byref(kms), C.byref(kbytes))
    lib.mr_ctx_profile(ctx.h, 0)
    it_us = kms.value / max(launches.value, 1) * 1e3
    it_bytes = kbytes.value / max(launches.value, 1)
    coll = ("IPC peer push" if shard.peer_active(ctx) else "RCCL") if world > 1 else "none (one rank)"
    t = torch.tensor([el, nnz, it_us, it_bytes], dtype=torch.float64)
    if dist is not None:
        mx, sm = t.clone(), t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        el, nnz, it_us, it_bytes = float(mx[0]), float(sm[1]), float(mx[2]), float(sm[3])
    dg.close()
    ctx.close()
    edges = 25.0 * (2.0 * nnz + E) * steps
    return {"workload": f"C4: one {C4_OPS}-op / {C4_TRACES}-trace graph (fp64, anomaly preference) sharded by "
                        f"trace over {world} GPU(s); a step = one whole trace_pagerank",
            "value": round(edges / el / 1e9, 3), "unit": "GTEPS", "ms_per_step": round(el / steps * 1e3, 4),
            "steps": steps, "warmup": warmup, "n_gpus": world, "scaling": "strong", "nnz": int(nnz),
            "call_edges": int(E), "traces_per_rank": C4_TRACES // world,
            "iteration_us_max_rank": round(it_us, 3),
            "iteration_frac": round(it_bytes / (it_us * 1e-6) / 1e9 / HBM_PEAK_GBS / world, 4) if it_us > 0 else None,
            "all_reduce": coll,
            "what": "iteration_us_max_rank: the slowest rank's HIP-event time of one iteration's launches (walk, "
                    "column sums, all-reduce, finish); iteration_frac: SURVEY B_iter of the whole graph / that "
                    "time / (N x 8 TB/s)"}


def run_merged_leg(out, run_all, ctx, lib, steps, nnz_w):
    """The run-merged walk (MR_TR_MERGE=1, read per call): runs of identical traces -- adjacent
    positions of one kind class in the layout -- share one id rotation and k_tr_a walks each run
    by its head (the run's adds as one integer add of r x X, the tails' r' by shuffle; bitwise the
    per-trace walk).  That is SURVEY 8(f)4's kind compression inside the walk, so it is reported
    here, under its own keys, and never in `value` / `roofline.frac`: the same windows, steps of
    the same shape, this rank only."""
    import ctypes as C

    os.environ["MR_TR_MERGE"] = "1"
    try:
        run_all(1)   # (warm-up: the windows' graphs re-prepared with run rotations)
        ctx.sync()
        lib.mr_ctx_profile(ctx.h, 1)
        ts = time.perf_counter()
        edges, n_win, _ = run_all(steps)
        ctx.sync()
        el = time.perf_counter() - ts
        launches, kms, kbytes = C.c_int64(), C.c_double(), C.c_double()
        lib.mr_ctx_prof_read(ctx.h, C.byref(launches), C.byref(kms), C.byref(kbytes))
        lib.mr_ctx_profile(ctx.h, 0)
    finally:
        os.environ.pop("MR_TR_MERGE", None)
    avg_ms = kms.value / max(launches.value, 1)
    bpl = kbytes.value / max(launches.value, 1)
    ach = bpl / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    b16 = bpl - 2.0 * nnz_w * n_win * 25.0 / max(launches.value, 1)
    out["value_run_merged"] = round(edges / el / 1e9, 3)
    out["windows_per_s_run_merged"] = round(n_win / el, 3)
    out["roofline"]["run_merged"] = {
        "achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
        "u16_frac": round(b16 / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if avg_ms > 0 else None,
        "avg_launch_us": round(avg_ms * 1e3, 3), "launches": launches.value, "ms_per_step": round(el / steps * 1e3, 3),
        "what": f"MR_TR_MERGE=1, {steps} steps of the same windows: a run of identical traces walked by its head "
                "(kind compression inside the walk, SURVEY 8(f)4) -- the bytes and edges are still counted per "
                "trace, so these fractions credit avoided work; value_run_merged is its GTEPS"}


def isolated_group_roofline(ctx, group, prec, reps=3):
    """roofline.isolated: the timed line's iteration pair measured while builds of other windows run
    beside it on the auxiliary streams (the pipeline's contention included); here one call of ONE
    group (c2: 128 windows), whose builds finish before its PageRanks start, so the group's
    iterations run alone -- the kernel's own share of the HBM roofline."""
    import ctypes as C

    from microrank_amd import _lib
    from microrank_amd.online_rca import rank_windows

    lib = _lib.load()
    pr = "fp32" if prec == _lib.MR_FP32 else "fp64"
    # one group of the whole call (the library otherwise keeps groups to half a call, so that a
    # call's builds overlap its PageRanks); MR_WIN_GROUP is read per call
    old = os.environ.get("MR_WIN_GROUP")
    os.environ["MR_WIN_GROUP"] = str(len(group))
    try:
        rank_windows(ctx, [w[:5] for w in group], precision=pr)
        ctx.sync()
        lib.mr_ctx_profile(ctx.h, 1)
        for _ in range(reps):
            rank_windows(ctx, [w[:5] for w in group], precision=pr)
        ctx.sync()
        launches, kms, kbytes = C.c_int64(), C.c_double(), C.c_double()
        lib.mr_ctx_prof_read(ctx.h, C.byref(launches), C.byref(kms), C.byref(kbytes))
        lib.mr_ctx_profile(ctx.h, 0)
    finally:
        if old is None:
            os.environ.pop("MR_WIN_GROUP", None)
        else:
            os.environ["MR_WIN_GROUP"] = old
    avg_ms = kms.value / max(launches.value, 1)
    achieved = (kbytes.value / max(launches.value, 1)) / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    return {"achieved": round(achieved, 1), "frac": round(achieved / HBM_PEAK_GBS, 4),
            "avg_launch_us": round(avg_ms * 1e3, 3), "launches": launches.value,
            "bytes_per_launch": round(kbytes.value / max(launches.value, 1)),
            "what": f"one {len(group)}-window group per mr_windows_batch call (its builds done before its 25 iterations): "
                    "the iteration launches without concurrent builds; the line's frac is the same launches "
                    "inside the timed 256-window calls, beside the next group's builds"}


def c4_leg_guarded(hg, world, rank, dist, line, limit_s=240.0):
    """c4_leg_run behind a watchdog: a leg that raises becomes {"error": ...} (ranks stay in step:
    every rank raises on a library error the ranks agreed on); a leg still running after limit_s
    (a rank lost inside a collective) prints the headline line on rank 0 (with the leg's error in
    it) and ends the process with exit status 3, so the hang is visible to the driver as a failure
    while the line stays on stdout."""
    import threading

    if isinstance(hg, Exception):
        return {"error": f"generation: {type(hg).__name__}: {hg}"}

    def expire():
        if line is not None:
            line["c4_sharded"] = {"error": f"timed out after {limit_s:.0f} s"}
            emit(line)
        print(f"[bench] c4_sharded leg hung for {limit_s:.0f} s: exiting with status 3", file=sys.stderr, flush=True)
        os._exit(3)

    wd = threading.Timer(limit_s, expire)
    wd.daemon = True
    wd.start()
    try:
        return c4_leg_run(hg, world, rank, dist)
    except Exception as e:
        return {"error": f"{type(e).__name__}: {e}"}
    finally:
        wd.cancel()


def run_sweep(args):
    """SURVEY 8(f) f3 -- the driver's window sweep over a long resident span stream (C3-shaped
    traffic: 500 ops, 20k traces per 5 minutes).  A step is the whole online_anomaly_detect_RCA
    chain (online_rca.py:161-216) on the device: one mr_detect_sweep pass for every window start,
    the chain walk, ONE mr_windows_batch over its triggered windows.  Beside it: every 1-minute
    sliding window of the stream ranked over the same resident table (C3's "sliding windows"), and
    the window-by-window loop of round 1 (mr_detect + mr_rca_window per visited window)."""
    import ctypes as C

    from microrank_amd import _lib, synth
    from microrank_amd._lib import ptr
    from microrank_amd.online_rca import rank_windows, sweep_chain, sweep_plan, sweep_rank
    from microrank_amd.preprocess_data import DeviceSpans

    minutes = args.sweep_minutes
    n_tr = int(4000 * minutes)
    topo = synth.make_topology(500, 1234)
    normal = synth.gen_spans(topo, 20_000, 1235, branch=1.9, p_max=0.8, names=False)
    stream = synth.gen_spans(topo, n_tr, 1236, minutes=minutes / 0.97, branch=1.9, p_max=0.8, names=False,
                             fault_op=synth.fault_op_of(topo), fault_frac=args.sweep_fault, fault_ms=6000.0)
    ctx = _lib.default_context()
    a3, ok = slo_from_gpu(ctx, normal)
    dev = DeviceSpans(ctx, stream)
    t_begin, t_end = int(stream.tstart.min()), int(stream.tend.max())
    step_n, step_a = 5 * 60 * 10**9, 4 * 60 * 10**9

    def driver_step():
        plan = sweep_plan(ctx, stream, dev, a3, ok, t_begin, t_end, step_n, step_a)
        ev = sweep_chain(plan)
        res = sweep_rank(plan, ev)
        return ev, res

    for _ in range(args.warmup):
        driver_step()
    ctx.sync()
    ts = time.perf_counter()
    for _ in range(args.steps):
        ev, res = driver_step()
    ctx.sync()
    dt = (time.perf_counter() - ts) / args.steps
    visited = sum(1 for e in ev if e[0] == "window")
    ranked = len(res)
    # the round-1 loop: the detector of each visited window, then mr_rca_window for the triggered ones
    lib = _lib.load()
    state = np.zeros(stream.n_traces, np.uint8)

    def loop_step():
        t, out = t_begin, 0
        na, nn, nin = C.c_int32(), C.c_int32(), C.c_int64()
        while t < t_end:
            rc = lib.mr_detect(ctx.h, dev.h, t, t + step_n, ptr(a3, C.c_double), ptr(ok, C.c_uint8),
                               ptr(state, C.c_uint8), C.byref(na), C.byref(nn), C.byref(nin))
            if rc == _lib.MR_ERR_VALUE and nin.value == 0:
                break
            ctx.check(rc, "mr_detect")
            trig = na.value > 0 and nn.value > 0
            if trig:
                run_window(ctx, dev, t, t + step_n, a3, ok, 0)
                out += 1
            t += step_n + (step_a if trig else 0)
        return out

    loop_step()
    ts = time.perf_counter()
    n_loop = loop_step()
    ctx.sync()
    dt_loop = time.perf_counter() - ts
    assert n_loop == ranked
    # every 1-minute sliding window of the stream, ranked in calls of 64 over the one resident table
    grain = 60 * 10**9
    starts = [t for t in range(t_begin, t_end - step_n + 1, grain)]
    wins = [(dev, t, t + step_n, a3, ok) for t in starts]
    rank_windows(ctx, wins[:64])
    ctx.sync()
    ts = time.perf_counter()
    n_ok = 0
    for i in range(0, len(wins), 64):
        n_ok += sum(1 for r in rank_windows(ctx, wins[i:i + 64]) if r[5] == _lib.MR_OK and r[1].size)
    ctx.sync()
    dt_slide = time.perf_counter() - ts
    return {"metric": "RCA driver sweep: windows ranked/sec (SURVEY 8(f) f3)", "value": round(ranked / dt, 2),
            "unit": "windows/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True, "scaling": "none", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic (seeded C3-shaped span stream, int-coded, resident in HBM)",
            "config": {"workload": f"online_anomaly_detect_RCA over {minutes:.0f} minutes of traffic: 500 ops, "
                                   f"{n_tr} traces, {stream.n_spans} spans, fault in {args.sweep_fault:.1%} of traces",
                       "windows_visited": visited, "windows_ranked": ranked, "window_starts_swept": int(plan_starts(t_begin, t_end))},
            "visited_per_s": round(visited / dt, 2),
            "window_loop": {"what": "round-1 loop: mr_detect per visited window + mr_rca_window per triggered one",
                            "ms": round(dt_loop * 1e3, 3), "windows_ranked_per_s": round(n_loop / dt_loop, 2),
                            "speedup_of_sweep": round(dt_loop / dt, 2)},
            "sliding": {"what": "every 1-minute window start of the stream ranked (mr_windows_batch, 64 per call, "
                                "one resident table)", "windows": len(wins), "ranked": n_ok,
                        "windows_per_s": round(len(wins) / dt_slide, 2)}}


def run_stream(args):
    """SURVEY 8(f) f3 online -- RCAStream over a C3-shaped string stream (500 ops, 4000 traces per
    minute, the reference's DataFrame schema) pushed in trace-aligned chunks of several sizes.  Per
    chunk size: the table update of one push on its own (device mode: mr_spans_append -- the chunk
    crosses PCIe, the resident rows are gathered and re-coded in HBM; host mode: pd.concat of the
    resident frame + a full re-ingest, the round-2 RCAStream) once the resident table has reached
    its steady size, and the whole stream's wall time through RCAStream in both modes (ranking
    included).  The device update should scale with the chunk, the host one with the table."""
    import contextlib
    import io
    import tempfile

    import pandas as pd

    from microrank_amd import _lib, synth
    from microrank_amd.online_rca import RCAStream
    from microrank_amd.preprocess_data import SpanStream, get_operation_slo, get_service_operation_list, span_table

    minutes = args.stream_minutes
    t_gen = time.perf_counter()
    ndf, adf = synth.stream_dataframes(500, int(4000 * minutes), 1301, minutes=minutes, branch=1.9, p_max=0.8,
                                       fault_ms=6000.0, fault_frac=0.0003)
    print(f"[bench] stream: {len(adf)} spans generated in {time.perf_counter() - t_gen:.1f} s", file=sys.stderr,
          flush=True)
    ctx = _lib.default_context()
    slo = get_operation_slo(get_service_operation_list(ndf), ndf)
    op_list = list(slo)
    t0 = adf["startTime"].min()
    window = pd.Timedelta(minutes=5)
    per_chunk = {}
    for cm in args.stream_chunks:
        bucket = ((adf["startTime"] - t0) // pd.Timedelta(minutes=cm)).to_numpy()
        cuts = np.flatnonzero(np.diff(bucket)) + 1
        bounds = np.concatenate([[0], cuts, [len(adf)]])
        chunks = [adf.iloc[bounds[i]:bounds[i + 1]] for i in range(len(bounds) - 1)]
        # steady state: the resident table holds the last 5 minutes + the chunk
        dev_ms, host_ms, res_spans = [], [], []
        st = SpanStream(ctx)
        resident = None
        for i, ch in enumerate(chunks):
            keep_from = ch["startTime"].min() - window
            ts = time.perf_counter()
            st.append(ch, int(keep_from.value))
            ctx.sync()
            t_dev = time.perf_counter() - ts
            ts = time.perf_counter()
            resident = ch if resident is None else pd.concat([resident[resident["startTime"] >= keep_from], ch],
                                                             ignore_index=True)
            span_table(resident, ctx)
            ctx.sync()
            t_host = time.perf_counter() - ts
            if ch["startTime"].min() - t0 >= window + pd.Timedelta(minutes=cm):
                dev_ms.append(t_dev * 1e3)
                host_ms.append(t_host * 1e3)
                res_spans.append(st.table.n_spans)
        st.close()
        # the whole stream through RCAStream, both modes (same printed output)
        walls, outs = {}, {}
        cwd = os.getcwd()
        with tempfile.TemporaryDirectory(dir="/tmp") as td:
            os.chdir(td)
            try:
                for mode in (True, False):
                    sink = io.StringIO()
                    ts = time.perf_counter()
                    with contextlib.redirect_stdout(sink):
                        s = RCAStream(slo, op_list, ctx=ctx, device_append=mode)
                        for ch in chunks:
                            s.push(ch)
                        s.close()
                    ctx.sync()
                    walls[mode] = time.perf_counter() - ts
                    outs[mode] = sink.getvalue()
            finally:
                os.chdir(cwd)
        n_chunk = [len(c) for c in chunks]
        per_chunk[f"{cm:g}min"] = {
            "chunks": len(chunks), "spans_per_chunk": int(np.mean(n_chunk)),
            "resident_spans": int(np.mean(res_spans)) if res_spans else None,
            "device_append_ms": round(float(np.median(dev_ms)), 2) if dev_ms else None,
            "host_concat_reingest_ms": round(float(np.median(host_ms)), 2) if host_ms else None,
            "stream_wall_s": {"device_append": round(walls[True], 3), "host_mode": round(walls[False], 3)},
            "windows_printed": outs[True].count("total_trace"),
            "same_output": outs[True] == outs[False]}
        print(f"[bench] stream {cm:g} min chunks: {per_chunk[f'{cm:g}min']}", file=sys.stderr, flush=True)
    best = per_chunk[f"{args.stream_chunks[0]:g}min"]
    return {"metric": "RCAStream push: table update ms per chunk (SURVEY 8(f) f3 online)",
            "value": best["device_append_ms"], "unit": "ms", "n_gpus": 1, "steps": len(args.stream_chunks),
            "warmup": 0, "ms_per_step": best["device_append_ms"], "higher_is_better": False, "scaling": "none",
            "vs_baseline": None, "dtype": "u8",
            "data": "synthetic reference-schema span DataFrames (strings), pushed in trace-start order",
            "config": {"workload": f"{minutes:g} minutes of C3-shaped traffic (500 ops, 4000 traces/min, "
                                   f"{len(adf)} spans), chunk sizes {args.stream_chunks} min",
                       "per_chunk": per_chunk}}


def run_dropin(args):
    """The north star's drop-in path, measured: the reference driver's window body
    (online_rca.py:167-201 -- system_anomaly_detect, get_pagerank_graph + trace_pagerank twice,
    calculate_spectrum_without_delay_list, the prints and result.csv) through the swapped imports
    (microrank_amd's drop-in modules, called on the reference's DataFrame exactly as the unchanged
    driver calls them: microrank_amd.online_rca._window_loop is that loop), at C1 and C2.  A step is
    one window on a resident DataFrame (its device span table cached after the first call); the
    reference's own C1 number is 0.43 windows/s (measured in the dev container)."""
    import contextlib
    import io
    import tempfile

    import pandas as pd

    from microrank_amd import online_rca as orca
    from microrank_amd import synth
    from microrank_amd.online_rca import _window_loop
    from microrank_amd.preprocess_data import get_operation_slo, get_service_operation_list

    # the window body's calls (online_rca.py:167-201), each timed on the host: the phase table
    phase_names = ("system_anomaly_detect", "get_pagerank_graph", "trace_pagerank",
                   "calculate_spectrum_without_delay_list", "_write_result")
    phase_ms = {}

    def timed(name, fn):
        def w(*a, **k):
            ts = time.perf_counter()
            try:
                return fn(*a, **k)
            finally:
                phase_ms[name] = phase_ms.get(name, 0.0) + (time.perf_counter() - ts) * 1e3
        return w

    sizes = {"C1": (40, 2000, 100), "C2": (args.ops, args.traces, 1234)}
    lines = {}
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        os.chdir(td)
        try:
            for name, (n_ops, n_tr, seed) in sizes.items():
                t_gen = time.perf_counter()
                ndf, adf = synth.window_dataframes(n_ops, n_tr, seed, branch=1.9, p_max=0.8, fault_ms=6000.0)
                print(f"[bench] dropin {name}: {len(adf)} spans generated in {time.perf_counter() - t_gen:.1f} s",
                      file=sys.stderr, flush=True)
                op_list = get_service_operation_list(ndf)
                slo = get_operation_slo(op_list, ndf)
                start = adf["startTime"].min()
                one = start + pd.Timedelta(1, unit="ns")   # the loop runs exactly the window at `start`
                sink = io.StringIO()
                ts = time.perf_counter()
                with contextlib.redirect_stdout(sink):
                    _window_loop(adf, slo, op_list, start, one)   # first call: ingests the DataFrame
                first_ms = (time.perf_counter() - ts) * 1e3
                ranked = "normal_list" in sink.getvalue()
                n = max(1, args.steps)
                ts = time.perf_counter()
                for _ in range(n):
                    with contextlib.redirect_stdout(io.StringIO()):
                        _window_loop(adf, slo, op_list, start, one)
                dt = (time.perf_counter() - ts) / n
                # the phase table: the same windows again with each drop-in call timed
                orig = {k: getattr(orca, k) for k in phase_names}
                phase_ms.clear()
                try:
                    for k in phase_names:
                        setattr(orca, k, timed(k, orig[k]))
                    ts = time.perf_counter()
                    for _ in range(n):
                        with contextlib.redirect_stdout(io.StringIO()):
                            _window_loop(adf, slo, op_list, start, one)
                    dt_p = (time.perf_counter() - ts) / n
                finally:
                    for k in phase_names:
                        setattr(orca, k, orig[k])
                phases = {k: round(phase_ms.get(k, 0.0) / n, 3) for k in phase_names}
                phases["other (loop, prints)"] = round(dt_p * 1e3 - sum(phases.values()), 3)
                lines[name] = {"windows_per_s": round(1.0 / dt, 3), "ms_per_window": round(dt * 1e3, 3),
                               "first_window_ms": round(first_ms, 1), "ranked": ranked,
                               "spans": int(len(adf)), "traces": int(adf["traceID"].nunique()), "ops": n_ops,
                               "phase_ms_per_window": phases}
                del ndf, adf
        finally:
            os.chdir(cwd)
    c1 = lines["C1"]["windows_per_s"]
    return {"metric": "drop-in RCA windows/sec through the reference driver's call sequence (north star)",
            "value": lines["C2"]["windows_per_s"], "unit": "windows/s", "n_gpus": 1, "steps": args.steps,
            "warmup": 1, "ms_per_step": lines["C2"]["ms_per_window"], "higher_is_better": True, "scaling": "none",
            "vs_baseline": None, "dtype": "f64",
            "data": "synthetic reference-schema DataFrames (strings), resident in host memory; device span table "
                    "cached per DataFrame after the first call",
            "config": {"workload": "online_rca.py:167-201 window body via the swapped imports, C2 (C1 beside)",
                       "C1": lines["C1"], "C2": lines["C2"]},
            "reference_cpu": {"C1_windows_per_s": 0.43, "source": "BASELINE.md / SURVEY 6 (reference Python, 1 core)",
                              "speedup_C1": round(c1 / 0.43, 1)}}


def plan_starts(t_begin, t_end, grain=60 * 10**9):
    return -(-(t_end - t_begin) // grain)


def run_ingest(args):
    """SURVEY 8(f) f2 -- span ingest: the C2 window's reference-schema DataFrame (strings) into
    the device span table.  A step is mr_spans_ingest on the DataFrame's Arrow string buffers
    (host memory: the copy over PCIe is inside the time) incl. the table's per-trace index; the
    CPU baseline is the pandas factorisation it replaces (SpanTable.from_dataframe)."""
    from microrank_amd import _lib, synth
    from microrank_amd.preprocess_data import DeviceSpans
    from microrank_amd.spans import SpanTable, arrow_columns

    topo, normal, abnormal = synth.window_pair(args.ops, args.traces, 1234, branch=1.9, p_max=0.8, fault_ms=6000.0)
    df = synth.to_dataframe(abnormal, topo, 1236)
    S = len(df)
    ts = time.perf_counter()
    arrays = arrow_columns(df)
    t_arrow = time.perf_counter() - ts
    ctx = _lib.default_context()
    for _ in range(args.warmup):
        t, d = DeviceSpans.ingest(ctx, df, arrays)
        d.close()
    ctx.sync()
    ts = time.perf_counter()
    for _ in range(args.steps):
        t, d = DeviceSpans.ingest(ctx, df, arrays)
        if _ != args.steps - 1:
            d.close()
    ctx.sync()
    dt = (time.perf_counter() - ts) / args.steps
    ts = time.perf_counter()
    host = SpanTable.from_dataframe(df)
    dt_host = time.perf_counter() - ts
    same = bool(np.array_equal(t.trace, host.trace) and np.array_equal(t.podop, host.podop) and
                np.array_equal(t.svcop, host.svcop) and list(t.podop_names) == list(host.podop_names))
    # end to end from the OTel CSV export: pyarrow reader + device ingest vs pandas read_csv +
    # rename + to_datetime + the factorisation (online_rca.py:221-248 and SpanTable.from_dataframe)
    import tempfile

    import pandas as pd

    from microrank_amd.spans import OTEL_RENAME, read_traces_csv

    csv_line = None
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        path = os.path.join(td, "traces.csv")
        df.rename(columns={v: k for k, v in OTEL_RENAME.items()}).to_csv(path, index=False)
        ts = time.perf_counter()
        dfa = read_traces_csv(path)
        t_read = time.perf_counter() - ts
        ts = time.perf_counter()
        ta, da = DeviceSpans.ingest(ctx, dfa, arrow_columns(dfa))
        ctx.sync()
        t_ing = time.perf_counter() - ts
        da.close()
        ts = time.perf_counter()
        dfp = pd.read_csv(path).rename(columns=OTEL_RENAME)
        dfp["startTime"] = pd.to_datetime(dfp["startTime"])
        dfp["endTime"] = pd.to_datetime(dfp["endTime"])
        t_pread = time.perf_counter() - ts
        ts = time.perf_counter()
        SpanTable.from_dataframe(dfp)
        t_pfact = time.perf_counter() - ts
        csv_line = {"what": "OTel CSV -> device span table: read_traces_csv (pyarrow) + mr_spans_ingest, "
                            "vs pandas read_csv + rename + to_datetime + factorisation",
                    "csv_MB": round(os.path.getsize(path) / 1e6, 1), "read_ms": round(t_read * 1e3, 1),
                    "ingest_ms": round(t_ing * 1e3, 1), "total_ms": round((t_read + t_ing) * 1e3, 1),
                    "pandas_read_ms": round(t_pread * 1e3, 1), "pandas_factorize_ms": round(t_pfact * 1e3, 1),
                    "speedup": round((t_pread + t_pfact) / (t_read + t_ing), 1)}
    str_bytes = sum(int(a.buffers()[2].size) if a.buffers()[2] is not None else 0 for a in arrays.values())
    in_bytes = str_bytes + 6 * 8 * (S + 1) + 3 * 8 * S
    d.close()
    return {"metric": "span ingest: spans/sec, strings -> device span table (SURVEY 8(f) f2)",
            "value": round(S / dt / 1e6, 3), "unit": "Mspans/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True, "scaling": "none",
            "vs_baseline": None, "dtype": "u8/int64", "data": "synthetic (C2 window as the reference's string schema)",
            "config": {"workload": f"C2 window DataFrame: {S} spans, {abnormal.n_traces} traces, {len(host.podop_names)} "
                                   f"pod-ops; input {in_bytes / 1e6:.1f} MB of Arrow buffers in host memory",
                       "pcie_inclusive": True},
            "arrow_ms": round(t_arrow * 1e3, 3), "codes_equal_host": same, "csv": csv_line,
            "input_GBps": round(in_bytes / dt / 1e9, 2),
            "cpu_baseline": {"value": round(S / dt_host / 1e6, 3), "unit": "Mspans/s", "cores": 1, "kind": "port",
                             "sample": "SpanTable.from_dataframe (pandas factorize of the same DataFrame), once",
                             "ms": round(dt_host * 1e3, 1)}}


# The driver reads ONE JSON line from stdout, but libraries write there too (the gloo rendezvous'
# "connected to N peer ranks", RCCL's version banner at communicator init): fd 1 is pointed at
# stderr for the run and the line goes to the original stdout.
_LINE_OUT = None


def claim_stdout():
    global _LINE_OUT
    if _LINE_OUT is None:
        sys.stdout.flush()
        fd = os.dup(1)
        os.dup2(2, 1)
        _LINE_OUT = os.fdopen(fd, "w")


def emit(obj):
    out = _LINE_OUT if _LINE_OUT is not None else sys.stdout
    out.write(json.dumps(obj) + "\n")
    out.flush()


def main():
    claim_stdout()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--precision", choices=["fp64", "fp32"], default=None,
                    help="default fp64 (c2, c4), fp32 (c5: BASELINE configs[4])")
    ap.add_argument("--ops", type=int, default=1000)
    ap.add_argument("--traces", type=int, default=200_000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--streams", type=int, default=None,
                    help="c2: windows per step (default 64: one mr_windows_batch call; --streams-mode: 8 contexts "
                         "/ streams / host threads, one window each); c3: windows per batch call (default 256)")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 PMC passes for roofline.traffic")
    ap.add_argument("--streams-mode", action="store_true",
                    help="c2/c3: W contexts + W host threads, one mr_rca_window per window (instead of mr_windows_batch)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--config", choices=["c2", "c3", "c4", "c5", "sweep", "stream", "ingest", "dropin"], default="c2",
                    help="c2: RCA windows (default, weak scaling); c3: a batch of --c3-windows 500-op / 20k-trace "
                         "windows split over the ranks (strong scaling); c4 / c5: one trace-sharded graph (strong "
                         "scaling; c5 = 100k ops / 100M traces fp32, the wide fused iteration); sweep: the driver's "
                         "window sweep over a long stream (f3); ingest: strings -> device span table (f2); "
                         "dropin: the reference driver's window body through the drop-in modules (C1, C2)")
    ap.add_argument("--sweep-minutes", type=float, default=240.0, help="sweep: minutes of traffic in the stream")
    ap.add_argument("--stream-minutes", type=float, default=30.0, help="stream: minutes of traffic pushed")
    ap.add_argument("--stream-chunks", type=float, nargs="+", default=[0.5, 1.0, 2.0, 5.0],
                    help="stream: chunk sizes in minutes (the first one is the headline)")
    ap.add_argument("--sweep-fault", type=float, default=0.00005, help="sweep: fraction of traces hit by the fault")
    ap.add_argument("--c3-windows", type=int, default=4096, help="c3: windows in the whole batch (all ranks)")
    ap.add_argument("--c3-distinct", type=int, default=4,
                    help="c3: distinct seeded windows resident per stream (the batch cycles through them)")
    ap.add_argument("--c4-ops", type=int, default=None, help="c4/c5 op count (default 10k / 100k)")
    ap.add_argument("--c4-traces", type=int, default=None, help="c4/c5 trace count over all ranks (10M / 100M)")
    ap.add_argument("--from-spans", action="store_true",
                    help="c4/c5: each rank holds a span shard and a step includes the K1 graph build (mr_graph_build_sharded)")
    ap.add_argument("--shard-of", type=int, default=1,
                    help="c4/c5 --from-spans at N=1: rank 0's share of a K-GPU deployment (c5: 12.5M of the 100M traces "
                         "at K=8), built and ranked on this GPU")
    ap.add_argument("--no-side", action="store_true",
                    help="c2/c3: the timed steps only -- no single-window latency, kind-compressed probe or "
                         "c4_sharded leg (rocprofv3 kernel tables of the timed shape alone)")
    ap.add_argument("--no-c4-leg", action="store_true", help="c2: skip the c4_sharded leg of the default line")
    ap.add_argument("--dump-maps", default=None,
                    help="write /proc/self/maps here after the warm-up (resolving native stack frames of a crash)")
    ap.add_argument("--c2-distinct", type=int, default=None,
                    help="c2: distinct seeded windows per step (default: every window of the step distinct)")
    args = ap.parse_args()
    if args.streams is None:
        # c3: a 4096-window batch in calls of 2048 (r04: 256 / 512 / 1024 / 2048 / 4096 windows per
        # call 26.0-26.6k / 28.4-28.6k / 29.2-30.1k / 30.1k / 29.2-30.3k windows/s, profiles/r04aa);
        # c2: calls of 256 (r04: 64 / 128 / 256 -> 4785 / 5269 / 6005-6091 windows/s, profiles/r04y)
        # -- the first group's build and the last group's iterations, which nothing overlaps,
        # spread over more windows
        args.streams = 8 if args.streams_mode else (2048 if args.config == "c3" else 256)
    if args.precision is None:
        args.precision = "fp32" if args.config == "c5" else "fp64"
    if args.c4_ops is None:
        args.c4_ops = 100_000 if args.config == "c5" else 10_000
    if args.c4_traces is None:
        args.c4_traces = 100_000_000 if args.config == "c5" else 10_000_000
    if args.config == "c3":   # BASELINE configs[2]: 500 ops / 20k traces per window
        args.ops, args.traces = 500, 20_000
        if "--steps" not in sys.argv:
            args.steps = 3
        if "--warmup" not in sys.argv:
            args.warmup = 1

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # PMC passes first, in child processes, before this process initialises the GPU
    traffic = None
    if world == 1 and not args.pmc_child and not args.no_traffic and args.config not in ("sweep", "stream", "ingest", "dropin"):
        traffic = pmc_traffic(args, timeout_s=240 if args.config in ("c2", "c3") else 400)
    dist = None
    if world > 1:
        import torch.distributed as dist  # control plane only: barrier + max over ranks (gloo, host)

        dist.init_process_group("gloo")
    os.environ.setdefault("MICRORANK_DEVICE", str(local))
    if args.config in ("sweep", "stream", "ingest", "dropin"):   # single-GPU supplementary lines (f2 / f3 / drop-in)
        if args.config in ("ingest", "dropin") and "--steps" not in sys.argv:
            args.steps, args.warmup = 5, 1
        if args.config == "sweep" and "--steps" not in sys.argv:
            args.steps, args.warmup = 3, 1
        out = {"sweep": run_sweep, "stream": run_stream, "ingest": run_ingest, "dropin": run_dropin}[args.config](args)
        emit(out)
        return
    if args.config in ("c4", "c5"):
        out = run_c4(args, world, rank, dist)
        if out is not None and traffic is not None:
            out["roofline"]["traffic"] = round(traffic["fetch"] + traffic["write"])
            out["roofline"]["traffic_detail"] = {
                "fetch_bytes": round(traffic["fetch"]), "write_bytes": round(traffic["write"]),
                "source": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) / WRITE_SIZE, per iteration (A + B launches)"}
        if out is not None:
            add_pmc_frac(out, traffic)
        if out is not None and not args.pmc_child:
            emit(out)
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return

    from microrank_amd import _lib
    from microrank_amd.preprocess_data import DeviceSpans

    # W independent windows per rank, each on its own context (HIP stream) and host thread: the
    # windows' small launches and host round trips overlap on the GPU (C3's data-parallel windows
    # within one device).  A step ranks all W windows.
    W = max(1, args.streams)
    dev_id = int(os.environ["MICRORANK_DEVICE"])
    batch = not args.streams_mode
    c2_tabs = None
    c4_hg = None   # the c4_sharded leg's shard (default line only), generated before the GPU is touched
    if (args.config == "c2" and batch and not args.pmc_child and not args.no_side and not args.no_c4_leg
            and not os.environ.get("MR_BENCH_NO_C4_LEG")):
        try:
            c4_hg = c4_leg_generate(world, rank)
        except Exception as e:   # (a side leg never sinks the line)
            c4_hg = e
    if batch and args.config == "c2":   # distinct windows, generated before the GPU is touched
        nd = W if args.c2_distinct is None else max(1, min(W, args.c2_distinct))
        t_gen = time.perf_counter()
        c2_tabs = c2_windows(nd, args.ops, args.traces, rank)
        print(f"[bench] rank {rank}: {nd} distinct C2 windows generated in {time.perf_counter() - t_gen:.1f} s",
              file=sys.stderr, flush=True)
    # batch (default): one context; a step is ONE mr_windows_batch call over W windows (their
    # detectors / builds / spectra on the library's auxiliary streams, their PageRanks sharing
    # each iteration's launches).  --streams-mode: W contexts driven by W host threads, one
    # mr_rca_window call per window (round-1 design, kept for A/B).
    ctxs = [_lib.default_context()] + ([] if batch else [_lib.Context(dev_id) for _ in range(W - 1)])
    # c2 (batch): W distinct seeded windows of one system, each its own span table resident in HBM
    # (one 5-minute window of 200k traces each), ranked by one mr_windows_batch call per step.
    # c2 --streams-mode: the same window's spans on every context (separate HBM copies).
    # c3: D distinct seeded windows per context; the rank's share of the batch cycles through them.
    D = max(1, args.c3_distinct) if args.config == "c3" else 1
    wins = [[] for _ in range(1 if batch else W)]   # per context: [(dev, t0, t1, a3, ok, abnormal)]
    if c2_tabs is not None:
        normal, tabs = c2_tabs
        a3, ok = slo_from_gpu(ctxs[0], normal)   # one SLO period; every table has the topology's codes
        for i, abnormal_i in enumerate(tabs):
            t0 = int(abnormal_i.tstart.min())
            dev_i = DeviceSpans(ctxs[0], abnormal_i)
            if i:   # host copy no longer needed (window 0's feeds the CPU baseline): ~140 MB a window
                dev_i.table = None
                tabs[i] = None
            wins[0].append((dev_i, t0, t0 + 5 * 60 * 10**9, a3, ok, abnormal_i if i == 0 else None))
            del abnormal_i
        abnormal, topo = tabs[0], None
        D = 0
    for d in range(D):
        seed = 1234 + 7919 * rank + 104729 * d
        if d == 0 or args.config == "c3":
            topo, normal, abnormal = make_window(seed, args.ops, args.traces)
        t0 = int(abnormal.tstart.min())
        for ci in range(min(W, 8) if batch and args.config == "c3" else W):   # c3 batch: 8 x D distinct windows
            cx = ctxs[0] if batch else ctxs[ci]
            if batch and ci > 0 and args.config != "c3":   # c2: W copies of the one window
                wins[0].append(wins[0][0])
                continue
            if args.config == "c3" and D * W > 1:
                # distinct windows on every context too (one generator call per (context, d))
                if ci > 0:
                    topo, normal, abnormal = make_window(seed + 31 * ci, args.ops, args.traces)
                    t0 = int(abnormal.tstart.min())
            a3, ok = slo_from_gpu(cx, normal)
            dev = DeviceSpans(cx, abnormal)          # window spans resident in HBM from here on
            wins[0 if batch else ci].append((dev, t0, t0 + 5 * 60 * 10**9, a3, ok, abnormal))
    del topo, normal
    c2_tabs = None
    ctx = ctxs[0]
    dev0, t0, t1, a3, ok, abnormal = wins[0][0]
    prec = _lib.MR_FP32 if args.precision == "fp32" else _lib.MR_FP64
    if args.config == "c3":
        # this rank's share of the batch, dealt round-robin over its contexts
        share = args.c3_windows // world + (1 if rank < args.c3_windows % world else 0)
        per_ctx = [len(range(ci, share, W)) for ci in range(W)] if not batch else None
    else:
        share, per_ctx = None, None

    def barrier():
        for cx in ctxs:
            cx.sync()
        if dist is not None:
            dist.barrier()

    step_times = []   # (batch mode) wall time of each step of the last run_all, ms

    def run_all(n):
        """n steps; (edges, windows, the first window's last result).  c2: a step is W windows;
        c3: a step is the rank's share of the batch."""
        if batch:
            from microrank_amd.online_rca import rank_windows

            pool = wins[0]
            per_step = share if share is not None else W   # c2: W windows, cycling the distinct ones
            res, first = [], None
            step_times.clear()
            for _ in range(n):
                ts_step = time.perf_counter()   # (each call returns its results: synchronous)
                for c0 in range(0, per_step, W):   # c3: calls of <= W windows
                    idx = range(c0, min(per_step, c0 + W))
                    out = rank_windows(ctx, [pool[j % len(pool)][:5] for j in idx],
                                       precision="fp32" if prec == _lib.MR_FP32 else "fp64")
                    for j, (codes, scores, na_, nn_, e_, st_) in zip(idx, out):
                        if st_ != 0:
                            raise RuntimeError(f"window {j}: status {st_}")
                        res.append(e_)
                        if j % len(pool) == 0:
                            first = (e_, codes, scores, na_, nn_)
                step_times.append((time.perf_counter() - ts_step) * 1e3)
            return sum(res), len(res), first

        def one(ci):
            cx, res = ctxs[ci], []
            cnt = n * (per_ctx[ci] if per_ctx is not None else 1)
            for j in range(cnt):
                dv, a, b, s3, sok, _ = wins[ci][j % len(wins[ci])]
                res.append(run_window(cx, dv, a, b, s3, sok, prec))
            return res
        if W == 1:
            outs = [one(0)]
        else:
            from concurrent.futures import ThreadPoolExecutor

            with ThreadPoolExecutor(max_workers=W) as ex:
                outs = list(ex.map(one, range(W)))
        # the last result of context 0's first window (the one the CPU baseline re-ranks)
        last0 = outs[0][(len(outs[0]) - 1) // len(wins[0]) * len(wins[0])] if outs[0] else None
        return sum(r[0] for o in outs for r in o), sum(len(o) for o in outs), last0

    run_all(args.warmup)
    if args.dump_maps:   # the libraries are all mapped by now (rocprofv3's tool included)
        with open("/proc/self/maps") as f, open(args.dump_maps, "w") as g:
            g.write(f.read())
    load = _lib.load()
    load.mr_ctx_profile(ctx.h, 1)
    barrier()
    t_start = time.perf_counter()
    edges, n_win, last = run_all(args.steps)
    barrier()
    elapsed = time.perf_counter() - t_start
    e, top, scores, na, nn = last
    import ctypes as C

    launches, kms, kbytes = C.c_int64(), C.c_double(), C.c_double()
    load.mr_ctx_prof_read(ctx.h, C.byref(launches), C.byref(kms), C.byref(kbytes))
    load.mr_ctx_profile(ctx.h, 0)
    if dist is not None:
        import torch

        t = torch.tensor([elapsed, float(edges), float(n_win)], dtype=torch.float64)
        mx = t.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = t.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed, edges_all, win_all = float(mx[0]), float(sm[1]), int(sm[2])
    else:
        edges_all, win_all = float(edges), n_win
    if rank != 0:
        if c4_hg is not None:   # (collective: every rank runs the leg)
            c4_leg_guarded(c4_hg, world, rank, dist, None)
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return
    avg_ms = kms.value / max(launches.value, 1)
    achieved = (kbytes.value / max(launches.value, 1)) / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    c3 = args.config == "c3"
    out = {
        "metric": "PageRank GTEPS + RCA windows ranked/sec at 1/2/4/8 MI355X; % HBM roofline",
        "value": round(edges_all / elapsed / 1e9, 3),
        "unit": "GTEPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if c3 else "weak",
        "vs_baseline": None,
        "dtype": "f64" if args.precision == "fp64" else "f32",
        "data": "synthetic (seeded Train-Ticket-like spans, int-coded, resident in HBM)"
                + (f"; {D * W} distinct windows per rank, the batch cycles through them" if c3 else
                   f"; {len(wins[0])} distinct windows per step (own seed and span table each)" if batch else ""),
        "config": {"workload": (f"C3 batch of {args.c3_windows} RCA windows ({args.ops} ops / {args.traces} traces "
                                f"each) over {world} GPU(s)" if c3 else
                                f"C2 RCA window: {args.ops} ops / {args.traces} traces per rank")
                               + ", detect + 2 graph builds + 2x25 PageRank iterations + DStar2 top-11",
                   "n_spans": int(abnormal.n_spans), "n_abnormal": na, "n_normal": nn,
                   "edges_per_window": int(edges // max(n_win, 1)),
                   "windows_per_step": (win_all // args.steps) if c3 else W,
                   "parallelism": (f"windows x{world} ranks, mr_windows_batch of {W} windows per call "
                                   f"(the PageRanks of a group of windows -- up to 32M traces, 16..128 windows -- share each "
                                   f"iteration's launches)") if batch
                                  else f"windows x{world} ranks x{W} streams"},
        "windows_per_s": round(win_all / elapsed, 3),
        "step_ms": ({"min": round(min(step_times), 3), "median": round(sorted(step_times)[len(step_times) // 2], 3),
                     "max": round(max(step_times), 3)} if step_times else None),
        "roofline": {"bound": "hbm", "kernel": ("one Jacobi iteration of a window group's graphs: the "
                                                "k_tr_a (+ k_fx_b) launch(es) over the graphs of one group (c2: 256 graphs of 128 "
                                                "windows; c3: 256 graphs of 128, one launch per iteration: the last "
                                                "block of each graph finishes it)") if batch else
                                               ("one Jacobi iteration: k_tr_a + k_fx_b (fused path)"
                                                + (f", stream 0 of {W} concurrent windows" if W > 1 else "")),
                     "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": None if traffic is None else round(traffic["fetch"] + traffic["write"]),
                     "traffic_detail": traffic and {"fetch_bytes": round(traffic["fetch"]),
                                                    "write_bytes": round(traffic["write"]),
                                                    "source": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) / WRITE_SIZE, "
                                                              "per iteration (A + B launches)"},
                     "avg_launch_us": round(avg_ms * 1e3, 3), "launches": launches.value,
                     "bytes_per_launch": round(kbytes.value / max(launches.value, 1))},
    }
    if args.pmc_child:
        return
    # SURVEY 8(d) window bytes: 52 S (the span columns once) + per graph build 24 S read + 4 nnz +
    # 4 T written + the window's PageRank iterations (the live per-iteration byte counts above)
    S = int(abnormal.n_spans)
    nnz_w = max(0.0, (edges // max(n_win, 1)) / 25.0) / 2.0   # 2 nnz + E per iteration, E << nnz
    bytes_w = 52.0 * S + 2 * 24.0 * S + 4.0 * nnz_w + 4.0 * (na + nn) + kbytes.value / max(n_win, 1)
    out["window_roofline"] = {"bytes_per_window": round(bytes_w), "achieved": round(bytes_w * n_win / elapsed / 1e9, 1),
                              "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": round(bytes_w * n_win / elapsed / 1e9 / HBM_PEAK_GBS, 4),
                              "formula": "52 S + 2 (24 S + 4 nnz + 4 T) + 25 B_iter per graph (SURVEY 8(d))",
                              "moved_bytes_per_window": round(bytes_w - 2.0 * nnz_w * 25.0)}   # (2-B ids in the walk)
    if launches.value and avg_ms > 0:   # the same launches on the bytes they move: 2-B op ids, not SURVEY's 4-B
        b16 = kbytes.value / launches.value - 2.0 * nnz_w * n_win * 25.0 / launches.value
        out["roofline"]["u16_ids"] = {"bytes_per_launch": round(b16), "achieved": round(b16 / (avg_ms * 1e-3) / 1e9, 1),
                                      "frac": round(b16 / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                      "what": "B_iter with 2 B per (trace, op) pair: k_tr_a reads u16 op ids"}
    add_pmc_frac(out, traffic)
    if args.no_side:
        add_copy_frac(out, ctx)
        emit(out)
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return
    if batch:
        try:   # kind compression inside the walk: its own leg, never the headline
            run_merged_leg(out, run_all, ctx, load, min(args.steps, 5), nnz_w)
        except Exception as e:  # a side metric never sinks the line
            out["roofline"]["run_merged"] = {"error": f"{type(e).__name__}: {e}"}
    if batch and args.config == "c2" and len(wins[0]) >= 128:
        try:   # the same iteration kernel with nothing beside it: ONE 128-window group per call
            out["roofline"]["isolated"] = isolated_group_roofline(ctx, wins[0][:128], prec)
        except Exception as e:  # a side metric never sinks the line
            out["roofline"]["isolated"] = {"error": f"{type(e).__name__}: {e}"}
    try:   # single-window latency: one window per mr_windows_batch call, nothing to overlap with
        from microrank_amd.online_rca import rank_windows

        one = [wins[0][0][:5]]
        pr = "fp32" if prec == _lib.MR_FP32 else "fp64"
        for _ in range(2):
            rank_windows(ctx, one, precision=pr)
        ctx.sync()
        lat = []
        for _ in range(15):
            ts = time.perf_counter()
            rank_windows(ctx, one, precision=pr)
            ctx.sync()
            lat.append((time.perf_counter() - ts) * 1e3)
        lat.sort()
        out["window_ms"] = {"median": round(lat[len(lat) // 2], 3), "min": round(lat[0], 3),
                            "what": "one window alone (W=1): detect + 2 graph builds + 2x25 iterations + spectrum, "
                                    "host wall time of one mr_windows_batch call"}
    except Exception as e:  # a side metric never sinks the line
        out["window_ms"] = {"error": f"{type(e).__name__}: {e}"}
    try:
        out["kind_compressed"] = kind_compressed_probe(ctx, dev0, t0, t1, a3, ok)
    except Exception as e:  # a side metric never sinks the line
        out["kind_compressed"] = {"error": f"{type(e).__name__}: {e}"}
    if c4_hg is not None:
        out["c4_sharded"] = c4_leg_guarded(c4_hg, world, rank, dist, out)
        c4_hg = None
    add_copy_frac(out, ctx)
    if not args.no_cpu and world == 1:   # the CPU baseline: rank 0 at N = 1 only
        try:
            cb, cres = cpu_baseline(abnormal, t0, t1, a3, ok)
            out["cpu_baseline"] = cb
            out["cpu_top_matches"] = bool(cres is not None and list(cres[0]) == list(top))
        except Exception as e:  # the baseline must never sink the GPU line
            out["cpu_baseline"] = {"value": None, "error": f"{type(e).__name__}: {e}"}
    emit(out)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

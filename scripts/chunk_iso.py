"""W distinct C2 windows (1000 ops / 200k traces; or OPS / TRACES) per mr_windows_batch call, N
calls: host wall time per call; under rocprofv3 --kernel-trace, `call_timeline.py` /
`win1_trace.py --analyze` split the trace per call (isolated kernel durations of one build chunk
when W <= the chunk size).
    python3 scripts/chunk_iso.py N W [OPS TRACES]"""
import sys
import time

sys.path.insert(0, ".")


def main(n, wn, ops=1000, traces=200_000):
    import bench
    from microrank_amd import _lib
    from microrank_amd.online_rca import rank_windows
    from microrank_amd.preprocess_data import DeviceSpans

    normal, abn = bench.c2_windows(wn, ops, traces, rank=0)
    ctx = _lib.default_context()
    s3, sok = bench.slo_from_gpu(ctx, normal)
    wins = []
    for ab in abn:
        d = DeviceSpans(ctx, ab)
        u0 = int(ab.tstart.min())
        wins.append((d, u0, u0 + 5 * 60 * 10**9, s3, sok))
    for _ in range(3):
        rank_windows(ctx, wins)
    ctx.sync()
    lat = []
    for _ in range(n):
        ts = time.perf_counter()
        rank_windows(ctx, wins)
        ctx.sync()
        lat.append((time.perf_counter() - ts) * 1e3)
    s = sorted(lat)
    print(f"W={wn} host ms: median {s[len(s) // 2]:.3f} min {s[0]:.3f}", flush=True)
    for w in wins:
        w[0].close()


if __name__ == "__main__":
    main(int(sys.argv[1]), int(sys.argv[2]), *[int(x) for x in sys.argv[3:5]])

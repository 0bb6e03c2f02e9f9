"""Cost of the drop-in span-table cache's exact "unchanged" check at C2 (VERDICT r3 item 8 asked
< 5 ms per lookup): one C2 window DataFrame, its device table built once, then timed cache hits.
    python3 scripts/cache_cost.py [ops] [traces]"""
import sys
import time

sys.path.insert(0, ".")


def main():
    from microrank_amd import synth
    from microrank_amd.preprocess_data import span_table

    n_ops = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    n_tr = int(sys.argv[2]) if len(sys.argv) > 2 else 200_000
    _, adf = synth.window_dataframes(n_ops, n_tr, 1234, branch=1.9, p_max=0.8, fault_ms=6000.0)
    kinds = {c: str(adf[c].dtype) for c in ("traceID", "spanID", "operationName", "duration")}
    ts = time.perf_counter()
    span_table(adf)
    first = (time.perf_counter() - ts) * 1e3
    lat = []
    for _ in range(20):
        ts = time.perf_counter()
        span_table(adf)
        lat.append((time.perf_counter() - ts) * 1e3)
    lat.sort()
    print(f"rows {len(adf)} dtypes {kinds}: first call (ingest) {first:.1f} ms; cache hit median "
          f"{lat[len(lat) // 2]:.2f} ms, min {lat[0]:.2f} ms", flush=True)


if __name__ == "__main__":
    main()

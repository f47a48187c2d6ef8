"""Summarise bench.py records (the driver's BENCH_*/SCALE_* files, or saved JSON lines) per N:
round time, per-kernel trace (train / Adam incl. the in-kernel xGMI exchange / eval /
all-reduce) and the plane companions (pull exchange, classic rounds), so a multi-GPU run
can be read without re-running it.

    python tools/scale_report.py SCALE_r05.json [BENCH_r05.json profiles/bench_*.json ...]

Any JSON document or JSON-lines file is accepted; every nested dict that looks like a
bench.py record (has "metric", "n_gpus" and "us_per_round") is reported.
"""
import json
import sys


def _records(obj):
    if isinstance(obj, dict):
        if {"metric", "n_gpus", "us_per_round"} <= obj.keys():
            yield obj
            return
        for v in obj.values():
            yield from _records(v)
    elif isinstance(obj, list):
        for v in obj:
            yield from _records(v)


def load(path):
    text = open(path).read()
    try:
        yield from _records(json.loads(text))
        return
    except json.JSONDecodeError:
        pass
    for line in text.splitlines():
        line = line.strip()
        if line.startswith("{"):
            try:
                yield from _records(json.loads(line))
            except json.JSONDecodeError:
                continue


def _trace(tr):
    if not isinstance(tr, dict):
        return "-"
    keys = [k for k in ("train", "adam", "eval", "allreduce", "eval_fedavg", "pack") if k in tr]
    return " ".join(f"{k} {tr[k]:.1f}" for k in keys) + f" | round {tr.get('round', float('nan')):.1f}"


def main(paths):
    recs = [r for p in paths for r in load(p)]
    if not recs:
        raise SystemExit("no bench.py records found")
    recs.sort(key=lambda r: (r.get("config", {}).get("model", ""), r["n_gpus"]))
    base = {}
    for r in recs:
        cfg = r.get("config", {})
        n = r["n_gpus"]
        us = r["us_per_round"]
        base.setdefault(cfg.get("model"), (n, us, r["value"]))
        n0, us0, v0 = base[cfg.get("model")]
        print(f"N={n} {cfg.get('round_design', '?'):24s} {cfg.get('data_plane', '?'):18s} "
              f"{us:8.2f} us/round  value {r['value']:.4g} (x{r['value'] / v0:.2f} vs N={n0})  "
              f"vs_baseline {r.get('vs_baseline') or float('nan'):.1f}  replicas {r.get('replicas_consistent')}")
        print(f"      kernels (eager trace, us/round, ~1.5 us marker cost each): {_trace(r.get('kernel_trace_us'))}")
        weak = r.get("weak_8000_rows_per_client")
        if isinstance(weak, dict):
            print(f"      weak 8000 rows/client: {weak.get('us_per_round', float('nan')):.2f} us/round")
        for name, c in (r.get("plane_companions") or {}).items():
            if not isinstance(c, dict):
                print(f"      companion {name}: {c}")
            elif "us_per_round" in c:
                print(f"      companion {name:8s} {c.get('round_design', '?'):24s} {c['us_per_round']:8.2f} us/round  "
                      f"{_trace(c.get('kernel_trace_us'))}")
            else:
                print(f"      companion {name}: {c}")


if __name__ == "__main__":
    main(sys.argv[1:])

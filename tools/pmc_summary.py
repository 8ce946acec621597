#!/usr/bin/env python3
"""Summarise two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; they cannot share a pass on
gfx950, MI355X_MICROARCH.md 'rocprofv3 PMC slots') into per-kernel HBM bytes per launch.

Corrections (MI355X_MICROARCH.md HBM section): rocprofv3 reports FETCH_SIZE / WRITE_SIZE in
KiB; on gfx950 FETCH_SIZE counts exactly half of the bytes of wide (16 B/lane) streaming reads,
so fetched bytes = 2 x FETCH_SIZE x 1024.  WRITE_SIZE is exact for 16 B/lane stores and float
atomics.  A calibration stream (tools/mb_stream, known bytes) can be passed to check both.

usage: pmc_summary.py <fetch_counter_collection.csv> <write_counter_collection.csv> <out.json>
                      [--calib <mb_fetch_counter_collection.csv>] [--routing <tools/pmc_decode.py json>] [--run b1|b8|b8i]
"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"^dsocr::", "", name)
    return name


def load(path, counter):
    """kernel -> counter values per dispatch, in dispatch order (values of one dispatch summed)."""
    per = defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        d = per[short(r["Kernel_Name"])]
        i = int(r["Dispatch_Id"])
        d[i] = d.get(i, 0.0) + float(r["Counter_Value"])
    return {k: [v[i] for i in sorted(v)] for k, v in per.items()}


def priced(kernels, fetch, write, routing):
    """The MoE launches of the routing file's plain generate (the last ones of each MoE kernel in dispatch
    order) priced one by one at their own distinct experts (bench.span_bytes): measured / algorithmic."""
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    cfgp = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "deepseek-ocr.rs_amd", "dsocr",
                        "configs", "deepseek-ocr.json")
    d = bench.lang_dims(json.load(open(cfgp)))
    B = routing["pages"]
    for k in kernels:
        kind = "moe_gateup" if k.startswith("moe_gateup_m") else ("moe_down" if k.startswith("moe_down_mm") else None)
        if kind is None or kind not in routing:
            continue
        seq = routing[kind]
        f, w = fetch.get(k, []), write.get(k, [])
        if len(f) < len(seq) or len(w) < len(seq):
            continue
        meas = [2.0 * 1024 * a + 1024 * b for a, b in zip(f[-len(seq):], w[-len(seq):])]
        alg = [bench.span_bytes(kind, d, B, 706, e, 0) for e in seq]
        kernels[k].update({"priced_launches": len(seq), "experts_mean": sum(seq) / len(seq),
                           "priced_hbm_bytes_per_launch": sum(meas) / len(meas),
                           "algorithmic_bytes_per_launch": sum(alg) / len(alg),
                           "traffic_over_algorithmic": sum(meas) / sum(alg)})


def main():
    fetch_csv, write_csv, out = sys.argv[1:4]
    fetch = load(fetch_csv, "FETCH_SIZE")
    write = load(write_csv, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        fk = sum(f) / len(f) if f else None
        wk = sum(w) / len(w) if w else None
        rd = 2.0 * fk * 1024 if fk is not None else None
        wr = wk * 1024 if wk is not None else None
        kernels[k] = {"launches": max(len(f), len(w)), "fetch_size_kib_mean": fk, "write_size_kib_mean": wk,
                      "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                      "hbm_bytes_per_launch": (rd or 0.0) + (wr or 0.0) if (rd is not None or wr is not None) else None}
    res = {"source": {"fetch": fetch_csv, "write": write_csv},
           "correction": "read = 2 x FETCH_SIZE[KiB] x 1024 (gfx950 half-count of wide streaming reads); write = WRITE_SIZE[KiB] x 1024",
           "kernels": kernels}
    if "--routing" in sys.argv:
        routing = json.load(open(sys.argv[sys.argv.index("--routing") + 1]))
        priced(kernels, fetch, write, routing)
        res["routing"] = {k: routing[k] for k in ("pages", "text_pages", "tokens")}
    if "--run" in sys.argv:
        run = sys.argv[sys.argv.index("--run") + 1]
        for v in kernels.values():
            v["run"] = run
    if "--calib" in sys.argv:
        cal = load(sys.argv[sys.argv.index("--calib") + 1], "FETCH_SIZE")
        res["calibration"] = {k: {"launches": len(v), "read_bytes_per_launch": 2.0 * 1024 * sum(v) / len(v)}
                              for k, v in cal.items()}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in sorted(kernels.items(), key=lambda kv: -(kv[1]["hbm_bytes_per_launch"] or 0))[:15]:
        print(f"{k[:70]:70s} n={v['launches']:6d} hbm/launch={(v['hbm_bytes_per_launch'] or 0) / 1e6:9.3f} MB")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Merge per-run PMC summaries (tools/pmc_summary.py outputs, each tagged --run) into one
profiles/rNN_pmc_traffic.json: table `kernels` = the one-page run (b1), `kernels_b8` = 8 text pages,
`kernels_b8i` = 8 image pages, `kernels_dots` = the dots tower; bench.py's pmc_traffic reads them by run tag.

usage: pmc_merge.py <out.json> run=summary.json [run=summary.json ...] [--carry <old rNN_pmc_traffic.json> dots]
"""
import json
import sys

TABLE = {"b1": "kernels", "b8": "kernels_b8", "b8i": "kernels_b8i", "dots": "kernels_dots"}


def main():
    out = sys.argv[1]
    res = {"correction": "read = 2 x FETCH_SIZE[KiB] x 1024 (gfx950 half-count of wide streaming reads); "
                         "write = WRITE_SIZE[KiB] x 1024", "source": {}}
    args = sys.argv[2:]
    carry = None
    if "--carry" in args:
        i = args.index("--carry")
        carry = (args[i + 1], args[i + 2:])
        args = args[:i]
    for a in args:
        run, path = a.split("=", 1)
        d = json.load(open(path))
        res["source"][run] = {"summary": path, "fetch": d["source"]["fetch"], "write": d["source"]["write"],
                              "routing": d.get("routing")}
        for v in d["kernels"].values():
            v["run"] = run
        res[TABLE[run]] = d["kernels"]
    if carry:
        old = json.load(open(carry[0]))
        for run in carry[1]:
            src = old.get(TABLE[run]) or {k: v for k, v in old.get("kernels", {}).items() if v.get("run") == run}
            res[TABLE[run]] = src
            res["source"][run] = {"carried_from": carry[0], "was": old.get("source", {}).get(run)}
    json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()

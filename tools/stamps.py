"""Dev: summarise per-block phase stamps written by profile_decode (DSOCR_STAMPS_OUT).

Layout per block: [wall clock at entry (100 MHz ticks), shader clock at phase 0..6].
Prints, over blocks: entry skew (wall), and per phase the median / p90 cycles since entry.
"""
import sys

import numpy as np


def main():
    a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 8).astype(np.int64)
    used = a[:, 0] != 0
    a = a[used]
    print(f"{len(a)} blocks stamped")
    wall = (a[:, 0] - a[:, 0].min()) * 10.0 / 1000.0  # us
    print(f"entry skew (us): p50 {np.median(wall):.2f} p90 {np.percentile(wall, 90):.2f} max {wall.max():.2f}")
    cyc = a[:, 1:]
    names = sys.argv[2].split(",") if len(sys.argv) > 2 else [f"p{i}" for i in range(7)]
    for i in range(1, 7):
        ok = cyc[:, i] != 0
        if not ok.any():
            continue
        d = (cyc[ok, i] - cyc[ok, 0]) / 2400.0  # us at 2.4 GHz nominal
        print(f"{names[i - 1] if i - 1 < len(names) else i:>12s}: n {ok.sum():5d} since entry p50 {np.median(d):6.2f} "
              f"p90 {np.percentile(d, 90):6.2f} max {d.max():6.2f} us")
    # end of every block on the wall clock: entry wall + cycles to last stamp
    last = np.array([r[r != 0][-1] - r[0] for r in cyc]) / 2400.0
    end = wall + last
    print(f"block end (us from first entry): p50 {np.median(end):.2f} max {end.max():.2f}")


if __name__ == "__main__":
    main()

"""Idle gaps of the GPU inside one C4 grid of a rocprofv3 kernel trace (development tool):
python tools/grid_gaps.py TRACE.csv [--min-us 30] [--window K]; grids are split at
score_kernel (one per grid); prints each gap with the kernels around it."""
import csv
import re
import sys


def short(n):
    return re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", "")).replace("void ", "")[-44:]


def main():
    path = sys.argv[1]
    mn = float(sys.argv[sys.argv.index("--min-us") + 1]) if "--min-us" in sys.argv else 30.0
    wk = int(sys.argv[sys.argv.index("--window") + 1]) if "--window" in sys.argv else -2
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                  for r in csv.DictReader(open(path)))
    cut = [i for i, r in enumerate(rows) if "score_kernel" in r[2]]
    wins = [rows[a + 1:b + 1] for a, b in zip(cut[:-1], cut[1:])]
    w = wins[wk]
    t0 = w[0][0]
    end = w[0][1]
    prev = w[0][2]
    tot = 0.0
    n = 0
    for s, e, name in w[1:]:
        if s > end:
            g = (s - end) / 1e3
            tot += g
            if g >= mn:
                n += 1
                print(f"{(end - t0) / 1e6:8.3f} ms  gap {g:7.1f} us  after {short(prev):44s} before {short(name)}")
        if e > end:
            end = e
            prev = name
    print(f"span {(end - t0) / 1e6:.3f} ms, idle {tot / 1e3:.3f} ms, {n} gaps >= {mn} us")


if __name__ == "__main__":
    main()

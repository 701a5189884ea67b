"""Detailed timeline of one window of a rocprofv3 kernel trace (development tool).

python tools/grid_window.py TRACE.csv T0_MS T1_MS [--gap 0.1]
Times are ms from the first dispatch.  Prints the dispatches of both queues in order, with
the idle gap before each one on the main queue, then busy totals per queue and kernel."""
import collections
import csv
import re
import sys


def short(n):
    n = re.sub(r"\(.*", "", n).replace("void ", "")
    return n[-48:]


def main():
    path, a, b = sys.argv[1], float(sys.argv[2]), float(sys.argv[3])
    gap_min = float(sys.argv[sys.argv.index("--gap") + 1]) if "--gap" in sys.argv else 0.1
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                     r["Queue_Id"]))
    rows.sort()
    t0 = rows[0][0]
    w = [r for r in rows if a <= (r[0] - t0) / 1e6 < b]
    qs = sorted(set(r[3] for r in w))
    last = {}
    busy = collections.defaultdict(float)
    tot = collections.defaultdict(lambda: [0.0, 0])
    union_end, union = None, 0.0
    for r in w:
        s, e = (r[0] - t0) / 1e6, (r[1] - t0) / 1e6
        g = s - last.get(r[3], s)
        last[r[3]] = max(last.get(r[3], e), e)
        busy[r[3]] += e - s
        tot[(r[3], short(r[2]))][0] += e - s
        tot[(r[3], short(r[2]))][1] += 1
        if union_end is None or s > union_end:
            union += e - s
            union_end = e
        elif e > union_end:
            union += e - union_end
            union_end = e
        if e - s > 0.15 or g > gap_min:
            print(f"{s:9.2f} +{e - s:6.2f} gap {g:5.2f} q{qs.index(r[3])} {short(r[2])}")
    span = (max(r[1] for r in w) - w[0][0]) / 1e6
    print(f"span {span:.2f} ms, GPU busy (union) {union:.2f} ms")
    for q in qs:
        print(f"queue {qs.index(q)}: {busy[q]:.2f} ms")
    for (q, k), (v, c) in sorted(tot.items(), key=lambda x: -x[1][0])[:25]:
        print(f"  q{qs.index(q)} {v:7.3f} ms {c:5d}x {k}")


if __name__ == "__main__":
    main()

"""Timeline of a rocprofv3 --kernel-trace CSV (development tool).

python tools/timeline.py TRACE.csv [--last-seconds S] [--match SUBSTR]
Reports, over the window (default: the last grid = dispatches after the last gap > 50 ms),
the wall span, the union of busy intervals (GPU busy), per-queue busy time, idle gaps, and the
per-kernel totals.  Kernel names are shortened to their first token.
"""
import argparse
import csv
import collections
import re


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "")
    return name[-60:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gap-ms", type=float, default=50.0)
    ap.add_argument("--windows", type=int, default=1, help="how many trailing windows")
    ap.add_argument("--split-on", default=None,
                    help="start a window at every dispatch whose name contains this")
    ap.add_argument("--skip-last", type=int, default=0, help="drop this many trailing windows")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         r["Queue_Id"]))
    rows.sort()
    # windows separated by gaps
    wins, cur = [], [rows[0]]
    last_end = rows[0][1]
    for r in rows[1:]:
        brk = (a.split_on in r[2]) if a.split_on else (r[0] - last_end > a.gap_ms * 1e6)
        if brk:
            wins.append(cur)
            cur = []
        cur.append(r)
        last_end = max(last_end, r[1])
    wins.append(cur)
    if a.skip_last:
        wins = wins[:-a.skip_last]
    for w in wins[-a.windows:]:
        t0 = w[0][0]
        t1 = max(r[1] for r in w)
        busy, s, e = 0, None, None
        for r in w:
            if s is None or r[0] > e:
                if s is not None:
                    busy += e - s
                s, e = r[0], r[1]
            else:
                e = max(e, r[1])
        busy += e - s
        print(f"window: {len(w)} dispatches, span {(t1 - t0) / 1e6:.2f} ms, GPU busy "
              f"{busy / 1e6:.2f} ms")
        perq = collections.defaultdict(int)
        tot = collections.defaultdict(lambda: [0, 0])
        for r in w:
            perq[r[3]] += r[1] - r[0]
            tot[short(r[2])][0] += r[1] - r[0]
            tot[short(r[2])][1] += 1
        for q, v in sorted(perq.items()):
            print(f"  queue {q}: {v / 1e6:.2f} ms of kernels")
        for k, (v, c) in sorted(tot.items(), key=lambda x: -x[1][0])[:30]:
            print(f"  {v / 1e6:8.3f} ms {c:5d}x  {k}")


if __name__ == "__main__":
    main()

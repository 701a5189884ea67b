"""Per-kernel breakdown of one design-matrix step in a rocprofv3 kernel trace (development
tool): python tools/dm_trace.py TRACE.csv"""
import collections
import csv
import re
import sys


def main():
    rows = []
    for r in csv.DictReader(open(sys.argv[1])):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    idx = [i for i, r in enumerate(rows) if "group_order_kernel" in r[2]]
    a, b = idx[-4], idx[-2]                  # the last full step (two groupings per step)
    w = rows[a:b]
    t0, t1 = w[0][0], max(r[1] for r in w)
    tot = collections.defaultdict(lambda: [0.0, 0])
    for s, e, n in w:
        nm = re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", ""))
        tot[nm][0] += (e - s) / 1e3
        tot[nm][1] += 1
    print(f"span {(t1 - t0) / 1e6:.3f} ms, busy {sum(e - s for s, e, _ in w) / 1e6:.3f} ms, "
          f"{len(w)} dispatches")
    for k, v in sorted(tot.items(), key=lambda x: -x[1][0]):
        print(f"{v[0]:9.1f} us {v[1]:4d} {k[-70:]}")


if __name__ == "__main__":
    main()

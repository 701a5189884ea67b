"""Per-workgroup timeline of one structured-Gram launch from the probe build
(variants/libsglm_trace.so, -DSGLM_LAGW_TRACE: s_memrealtime at block start / end, HW_ID, XCC_ID)
-- development tool.  python tools/lagw_trace.py PREFIX  ->  JSON summary per traced launch:
makespan, busy fraction of the CU slots over the makespan, mean block time per piece type and
the tail (time from the first CU going idle for good to the end)."""
import glob
import json
import sys

import numpy as np


def main():
    out = {}
    for path in sorted(glob.glob(sys.argv[1] + "_*.bin")):
        t = np.fromfile(path, dtype=np.uint64).reshape(-1, 4)
        t = t[t[:, 1] > 0]
        if t.size == 0:
            continue
        beg, end = t[:, 0].astype(np.int64), t[:, 1].astype(np.int64)
        t0 = beg.min()
        beg, end = (beg - t0) * 10, (end - t0) * 10              # ns (100 MHz clock)
        hw, xcc = (t[:, 2] & 0xffffffff).astype(np.int64), (t[:, 2] >> 32).astype(np.int64)
        cu = (xcc << 16) | ((hw >> 8) & 0xffff)                  # XCC, SE/SH/CU bits of HW_ID
        typ = (t[:, 3] & 0xffff).astype(np.int64)
        mk = int(end.max())
        slots = np.unique(cu)
        busy = float((end - beg).sum()) / (len(slots) * mk)
        last = np.array([end[cu == c].max() for c in slots])
        per_type = {int(k): round(float((end - beg)[typ == k].mean()) / 1e3, 1)
                    for k in np.unique(typ)}
        out[path.split("/")[-1]] = {
            "blocks": int(len(t)), "cus": int(len(slots)), "makespan_us": round(mk / 1e3, 1),
            "busy_frac": round(busy, 3),
            "cu_last_end_us_p10_p50_p90": [round(float(np.percentile(last, q)) / 1e3, 1)
                                           for q in (10, 50, 90)],
            "first_block_start_spread_us": round(float(np.sort(beg)[min(255, len(beg) - 1)]) / 1e3, 1),
            "block_us_by_type": per_type,
            "blocks_per_cu_max": int(np.bincount(np.searchsorted(slots, cu)).max()),
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

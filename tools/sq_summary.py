"""Per-launch SQ counter summary of one kernel from rocprofv3 --pmc passes (development tool).

python tools/sq_summary.py KERNEL_SUBSTRING OUT.json DIR [DIR ...] [--ms LAUNCH_MS]
Each DIR holds one pass's run_counter_collection.csv.  Counters are averaged over the kernel's
dispatches (every instantiation whose name contains the substring) and the derived ratios the
round-6 profiles quote are added: MFMA instructions (SQ_VALU_MFMA_BUSY_CYCLES / 32 for
v_mfma_f32_32x32x16_bf16), VALU / LDS / VMEM instructions per MFMA, MFMA-busy fraction of the
launch (over 1024 SIMDs at the clock given), LDS-wait and any-wait fractions of wave cycles
(quad-cycle units, MI355X_MICROARCH.md)."""
import csv
import collections
import json
import sys


def main():
    args = sys.argv[1:]
    ms = None
    if "--ms" in args:
        i = args.index("--ms")
        ms = float(args[i + 1])
        del args[i:i + 2]
    kern, out, dirs = args[0], args[1], args[2:]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = set()
    for d in dirs:
        for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
            if kern not in r["Kernel_Name"]:
                continue
            names.add(r["Kernel_Name"])
            per[(d, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    tot = collections.defaultdict(list)
    for (_, _), cs in per.items():
        for c, v in cs.items():
            tot[c].append(v)
    avg = {c: sum(v) / len(v) for c, v in tot.items()}
    nd = max(len(v) for v in tot.values()) if tot else 0
    der = {}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
        mf = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / 32.0
        der["mfma_per_launch"] = mf
        if "SQ_WAVES" in avg:
            der["mfma_per_wave"] = mf / avg["SQ_WAVES"]
        for c, k in (("SQ_INSTS_VALU", "valu_insts_per_mfma"), ("SQ_INSTS_LDS", "lds_insts_per_mfma"),
                     ("SQ_INSTS_VMEM_RD", "vmem_rd_insts_per_mfma")):
            if c in avg:
                der[k] = avg[c] / mf
        if ms:
            der["mfma_busy_frac_of_launch"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * 2.4e9 * ms * 1e-3)
            der["launch_ms_used"] = ms
            der["clock_ghz_assumed"] = 2.4
    if "SQ_WAVE_CYCLES" in avg:
        wc = avg["SQ_WAVE_CYCLES"]
        if "SQ_WAIT_INST_LDS" in avg:
            der["lds_wait_frac_of_wave_cycles"] = avg["SQ_WAIT_INST_LDS"] / wc
        if "SQ_WAIT_ANY" in avg:
            der["wait_any_frac_of_wave_cycles"] = avg["SQ_WAIT_ANY"] / wc
    json.dump({"kernel": kern, "instantiations": sorted(names), "dispatches": nd,
               "per_launch_avg": avg, "derived": der}, open(out, "w"), indent=1)
    print(json.dumps(der))


if __name__ == "__main__":
    main()

"""Interleaved A/B timing of kernel variants selected by environment switches that the library
reads per launch (development tool).  Box-to-box clocks differ by 20 %+, so variants are only
compared inside one process, alternating rounds, medians reported.

python tools/ab_micro.py eta|xtr [B,...] : C4 design (1M x 2000 event design), HIP events.
  eta : direction products sglm_gemv_eta_bits (SGLM_ETA_DIR=1 vs 0)
  eta3: exact (three-piece) products (SGLM_ETA_EXACT_STAGED=1 vs 0)
  xtr : gradient sglm_xtr_bits_packed (SGLM_XTR_NGW=2 vs 1, SGLM_XTR4=0 one-panel)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sabatinilab-glm_amd")]

VARIANTS = {
    "eta": [("dir", {"SGLM_ETA_DIR": "1"}), ("group", {"SGLM_ETA_DIR": "0"})],
    "etap": [("default", {"SGLM_ETA_PIPE": "1", "SGLM_ETA_PIPE_CFG": "0", "SGLM_ETA_DIR": "1"}),
             ("pipe28", {"SGLM_ETA_PIPE": "1", "SGLM_ETA_PIPE_CFG": "1"}),
             ("pipe42w2", {"SGLM_ETA_PIPE": "1", "SGLM_ETA_PIPE_CFG": "2"}),
             ("pipe44", {"SGLM_ETA_PIPE": "1", "SGLM_ETA_PIPE_CFG": "3"}),
             ("dir", {"SGLM_ETA_PIPE": "0", "SGLM_ETA_DIR": "1"}),
             ("group", {"SGLM_ETA_PIPE": "0", "SGLM_ETA_DIR": "0"})],
    "eta3": [("staged", {"SGLM_ETA_EXACT_STAGED": "1"}), ("group", {"SGLM_ETA_EXACT_STAGED": "0"})],
    "eta3p": [("pipe", {"SGLM_ETA_PIPE": "1", "SGLM_ETA3_CFG": "0"}),
              ("pipe_w2", {"SGLM_ETA_PIPE": "1", "SGLM_ETA3_CFG": "1"}),
              ("staged", {"SGLM_ETA_PIPE": "0", "SGLM_ETA_EXACT_STAGED": "1"})],
    "xtr": [("ngw2", {"SGLM_XTR4": "1", "SGLM_XTR_NGW": "2", "SGLM_XTR_PIPE": "0"}),
            ("pipe2", {"SGLM_XTR4": "1", "SGLM_XTR_NGW": "2", "SGLM_XTR_PIPE": "1"}),
            ("ngw1", {"SGLM_XTR4": "1", "SGLM_XTR_NGW": "1", "SGLM_XTR_PIPE": "0"}),
            ("pipe1", {"SGLM_XTR4": "1", "SGLM_XTR_NGW": "1", "SGLM_XTR_PIPE": "1"}),
            ("wpe2", {"SGLM_XTR4": "1", "SGLM_XTR_NGW": "3", "SGLM_XTR_PIPE": "0"}),
            ("pipe_wpe2", {"SGLM_XTR4": "1", "SGLM_XTR_NGW": "3", "SGLM_XTR_PIPE": "1"})],
    "xtrd": [("default", {}), ("pipe0", {"SGLM_XTR_PIPE": "0"})],
}


def main():
    import torch
    from sglm_hip import _lib, engine as E, synth
    what = sys.argv[1]
    sizes = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [120, 70]
    s = synth.make(N=1_000_000, m=50, L=20, family="poisson", rho=0.02, seed=0)
    d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    st = torch.cuda.current_stream().cuda_stream
    for B in sizes:
        rng = np.random.default_rng(B)
        slots = torch.arange(B, dtype=torch.int32, device="cuda")
        if what in ("eta", "etap", "eta3", "eta3p"):
            beta = torch.from_numpy(rng.normal(size=(B, d.P)).astype(np.float32)).cuda()
            out = torch.zeros((B, d.ld), dtype=torch.float32, device="cuda")
            work = torch.empty(_lib.query("sglm_eta_bits_work_bytes", d.P, B),
                               dtype=torch.uint8, device="cuda")

            def fn():
                _lib.call("sglm_gemv_eta_bits", d.rbits.data_ptr(), d.ld, d.P, beta.data_ptr(),
                          B, slots.data_ptr(), int(what in ("eta3", "eta3p")), out.data_ptr(),
                          work.data_ptr(), st)
        else:                                   # xtr, xtrd
            Bp = (B + 31) // 32 * 32
            rp = torch.zeros((3, Bp, d.ld), dtype=torch.bfloat16, device="cuda")
            rp[:, :B, :d.n] = torch.from_numpy(
                rng.normal(size=(3, B, d.n)).astype(np.float32)).cuda().to(torch.bfloat16)
            g = torch.zeros((B, d.P), dtype=torch.float64, device="cuda")
            work = torch.empty(_lib.query("sglm_xtr_bits_packed_work_bytes", d.P, B, d.ld),
                               dtype=torch.uint8, device="cuda")

            def fn():
                _lib.call("sglm_xtr_bits_packed", d.cbits_full().data_ptr(), d.ld, d.P, d.n,
                          rp.data_ptr(), B, slots.data_ptr(), g.data_ptr(), work.data_ptr(), st)
        times = {name: [] for name, _ in VARIANTS[what]}
        for rnd in range(6):
            for name, env in VARIANTS[what]:
                for k in ("SGLM_XTR4", "SGLM_XTR_NGW", "SGLM_XTR_PIPE"):
                    os.environ.pop(k, None)
                os.environ.update(env)
                fn()
                torch.cuda.synchronize()
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                if rnd:
                    times[name].append(e0.elapsed_time(e1) / 5)
        print(f"{what} B={B}: " + ", ".join(f"{k} {np.median(v):.3f} ms"
                                            for k, v in times.items()), flush=True)


if __name__ == "__main__":
    main()

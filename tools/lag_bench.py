"""Micro-benchmark of the gradient kernels on the C4 design (development tool):
sglm_lag_xtr (event occurrences) vs sglm_xtr_bits_packed (bit-plane MFMA) for B active fits,
HIP events on the launch stream, and the max |difference| of the two gradients."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sabatinilab-glm_amd")]


def main():
    import torch
    from sglm_hip import _lib, engine as E, synth
    s = synth.make(N=1_000_000, m=50, L=20, family="poisson", rho=0.02, seed=0)
    d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    lg = d.lag
    st = torch.cuda.current_stream().cuda_stream
    sizes = [int(v) for v in sys.argv[1].split(",")] if len(sys.argv) > 1 else [120, 16, 6]
    only = sys.argv[2] if len(sys.argv) > 2 else None
    for B in sizes:
        rng = np.random.default_rng(B)
        R = torch.zeros((B, d.ld), dtype=torch.float32, device="cuda")
        R[:, :d.n] = torch.from_numpy(rng.normal(size=(B, d.n)).astype(np.float32)).cuda()
        slots = torch.arange(B, dtype=torch.int32, device="cuda")
        g1 = torch.zeros((B, d.P), dtype=torch.float64, device="cuda")
        g2 = torch.zeros_like(g1)
        w1 = torch.empty(_lib.query("sglm_lag_xtr_work_bytes", d.P, lg.K, B, d.n),
                         dtype=torch.uint8, device="cuda")
        # the MFMA path's operand: R as three bf16 pieces, [3][ceil(B/32)*32][ld]
        Bp = (B + 31) // 32 * 32
        hi = R.to(torch.bfloat16)
        mid = (R - hi.float()).to(torch.bfloat16)
        lo = (R - hi.float() - mid.float()).to(torch.bfloat16)
        rp = torch.zeros((3, Bp, d.ld), dtype=torch.bfloat16, device="cuda")
        rp[0, :B], rp[1, :B], rp[2, :B] = hi, mid, lo
        w2 = torch.empty(_lib.query("sglm_xtr_bits_packed_work_bytes", d.P, B, d.ld),
                         dtype=torch.uint8, device="cuda")

        def lag():
            _lib.call("sglm_lag_xtr", lg.occ.data_ptr(), lg.tbeg.data_ptr(), lg.tend.data_ptr(),
                      lg.shifts.data_ptr(), lg.m, lg.K, lg.layout, lg.row0, d.n, d.P,
                      R.data_ptr(), d.ld, slots.data_ptr(), B, g1.data_ptr(), w1.data_ptr(), st)

        def bits():
            _lib.call("sglm_xtr_bits_packed", d.cbits_full().data_ptr(), d.ld, d.P, d.n,
                      rp.data_ptr(), B, slots.data_ptr(), g2.data_ptr(), w2.data_ptr(), st)
        out = {}
        for name, fn in (("lag", lag), ("bits", bits)):
            if only and name != only:
                out[name] = float("nan")
                continue
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            torch.cuda.synchronize()
            out[name] = e0.elapsed_time(e1) / 10
        diff = float((g1 - g2).abs().max() / g2.abs().max())
        print(f"B={B}: lag {out['lag']:.3f} ms, bits {out['bits']:.3f} ms, rel diff {diff:.2e}",
              flush=True)


if __name__ == "__main__":
    main()

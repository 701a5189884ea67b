"""Kernel micro-benchmarks on the C4 design shape (development tool, not the product bench).

python tools/bench_kernels.py [--fits B] [--rows N] [--variants 1,2] [--reps R]
Times each Gram variant with HIP events (interleaved rounds, one process) and checks the
variants agree; also times the Cholesky, eta and X^T R kernels at the same shape.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sabatinilab-glm_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fits", type=int, default=16)
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--m", type=int, default=50)
    ap.add_argument("--L", type=int, default=20)
    ap.add_argument("--variants", default="1,2")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--splits", type=int, default=1)
    ap.add_argument("--other", action="store_true", help="also time chol / eta / xtr")
    ap.add_argument("--masked", action="store_true",
                    help="also time sglm_syrk_masked with 20%% of 100-row trials held out")
    a = ap.parse_args()
    import torch
    from sglm_hip import _lib, engine as E, synth
    s = synth.make(N=a.rows, m=a.m, L=a.L, family="poisson", rho=0.02, seed=0)
    d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    B = a.fits
    g = torch.Generator(device="cuda").manual_seed(0)
    W = torch.zeros((B, d.ld), dtype=torch.float32, device="cuda")
    W[:, : d.n] = 0.2 + torch.rand((B, d.n), generator=g, device="cuda")
    fits = torch.arange(B, dtype=torch.int32, device="cuda")
    H = {v: torch.zeros((B, d.P, d.P), dtype=torch.float32, device="cuda") for v in
         [int(x) for x in a.variants.split(",")]}
    wb = _lib.query("sglm_syrk_work_bytes", d.P, B, a.splits)
    work = torch.empty(max(wb, 16), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    pa = d.p + 1
    nt = d.P // 256
    exec_flop = B * (nt * (nt + 1) // 2) * 256 * 256 * 2.0 * d.n
    alg_flop = B * float(d.n) * pa * (pa + 1)
    res = {"shape": {"n": d.n, "p": d.p, "P": d.P, "fits": B, "splits": a.splits}}
    times = {v: [] for v in H}

    def cbits_setup(mask, Wsrc):
        prob = E.Problem(d, [np.zeros(d.n)], [mask])
        cb = prob.compact(0)
        stride = max(64, (cb[1] + 63) // 64 * 64)
        wc = torch.zeros(B * stride, dtype=torch.bfloat16, device="cuda")
        desc = torch.tensor([[cb[0].data_ptr(), cb[1], wc.data_ptr() + 2 * k * stride,
                              0 if cb[2] is None else cb[2].data_ptr()] for k in range(B)],
                            dtype=torch.int64).cuda()
        _lib.call("sglm_gather_w", Wsrc.data_ptr(), d.ld, fits.data_ptr(), B, desc.data_ptr(),
                  cb[1], st)
        return prob, wc, desc

    if 6 in H:
        cb6 = cbits_setup(np.ones(d.n, np.uint8), W)
    for rep in range(a.reps + 1):
        for v in H:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if v == 6:
                _lib.call("sglm_syrk_cbits", cb6[2].data_ptr(), d.P, fits.data_ptr(), B, a.splits,
                          H[v].data_ptr(), work.data_ptr(), st)
            elif v == 3:
                _lib.call("sglm_syrk_bits", d.xbits.data_ptr(), d.ld, d.P, d.n, W.data_ptr(),
                          fits.data_ptr(), B, a.splits, H[v].data_ptr(), work.data_ptr(),
                          None, None, None, st)
            else:
                _lib.call("sglm_syrk_variant", v, d.xb.data_ptr(), d.ld, d.P, d.n, W.data_ptr(),
                          fits.data_ptr(), B, a.splits, H[v].data_ptr(), work.data_ptr(), st)
            e1.record()
            torch.cuda.synchronize()
            if rep:
                times[v].append(e0.elapsed_time(e1) / 1e3)
    if d.xbits is not None and 3 in H:
        pass
    for v in H:
        t = float(np.median(times[v]))
        res[f"syrk_v{v}"] = {"ms": t * 1e3, "exec_TFLOPs": exec_flop / t / 1e12,
                             "alg_TFLOPs": alg_flop / t / 1e12, "min_ms": min(times[v]) * 1e3}
    if a.masked:
        rng = np.random.default_rng(1)
        ntr = (d.n + 99) // 100
        m = np.repeat(rng.random(ntr) >= 0.2, 100)[: d.n].astype(np.uint8)
        prob = E.Problem(d, [np.zeros(d.n)], [m])
        Wm = W.clone()
        Wm[:, : d.n] *= torch.from_numpy(m.astype(np.float32)).cuda()
        goff = torch.zeros(B, dtype=torch.int64, device="cuda")
        gcnt = torch.full((B,), int(prob.group_count[0]), dtype=torch.int32, device="cuda")
        Hm = torch.zeros_like(H[list(H)[0]])
        use_bits = d.xbits is not None and 3 in H
        tm = []
        for rep in range(a.reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if use_bits:
                _lib.call("sglm_syrk_bits", d.xbits.data_ptr(), d.ld, d.P, d.n, Wm.data_ptr(),
                          fits.data_ptr(), B, a.splits, Hm.data_ptr(), work.data_ptr(),
                          prob.groups.data_ptr(), goff.data_ptr(), gcnt.data_ptr(), st)
            else:
                _lib.call("sglm_syrk_masked", d.xb.data_ptr(), d.ld, d.P, d.n, Wm.data_ptr(),
                          fits.data_ptr(), B, a.splits, Hm.data_ptr(), work.data_ptr(),
                          prob.groups.data_ptr(), goff.data_ptr(), gcnt.data_ptr(), st)
            e1.record()
            torch.cuda.synchronize()
            if rep:
                tm.append(e0.elapsed_time(e1) / 1e3)
        t = float(np.median(tm))
        rows = float(m.sum())
        res["syrk_masked"] = {"ms": t * 1e3, "train_rows": rows,
                              "groups_frac": float(prob.group_count[0]) * 8 / d.n,
                              "alg_TFLOPs": B * rows * pa * (pa + 1) / t / 1e12}
        if 6 in H:
            cbm = cbits_setup(m, Wm)
            H6 = torch.zeros_like(Hm)
            tm = []
            for rep in range(a.reps + 1):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                _lib.call("sglm_syrk_cbits", cbm[2].data_ptr(), d.P, fits.data_ptr(), B, a.splits,
                          H6.data_ptr(), work.data_ptr(), st)
                e1.record()
                torch.cuda.synchronize()
                if rep:
                    tm.append(e0.elapsed_time(e1) / 1e3)
            t = float(np.median(tm))
            up = torch.triu(torch.ones((d.P, d.P), dtype=torch.bool, device="cuda"))
            res["syrk_masked_v6"] = {"ms": t * 1e3,
                                     "alg_TFLOPs": B * rows * pa * (pa + 1) / t / 1e12,
                                     "maxrel_vs_masked": float(((H6[:, up] - Hm[:, up]).abs().max()
                                                                / Hm[:, up].abs().max()).item())}
    vs = list(H)
    if len(vs) > 1:
        up = torch.triu(torch.ones((d.P, d.P), dtype=torch.bool, device="cuda"))
        a0 = H[vs[0]][:, up]
        for v in vs[1:]:
            res[f"maxrel_v{v}_vs_v{vs[0]}"] = float(((H[v][:, up] - a0).abs().max() / a0.abs().max()).item())
    if a.other:
        bf = E._scratch().buf.get(B, d.P, d.ld, "cuda")
        bf.H.copy_(H[vs[-1]])
        dsh = torch.full((B, d.P), -1.0, dtype=torch.float32, device="cuda")
        dsh[:, : d.p] = 1e-2 * d.n
        dsh[:, d.p] = 0
        gvec = torch.randn((B, d.P), dtype=torch.float64, device="cuda")
        for name, fn in [
            ("chol", lambda: _lib.call("sglm_chol_solve_ex", bf.H.data_ptr(), d.P, fits.data_ptr(), B,
                                       gvec.data_ptr(), dsh.data_ptr(), bf.delta.data_ptr(),
                                       bf.info.data_ptr(), bf.frozen.data_ptr(), 1, B,
                                       bf.cwork.data_ptr(), st)),
            ("eta", lambda: d.eta(bf.beta, bf.eta)),
            ("xtr", lambda: _lib.call("sglm_xtr", d.xg.data_ptr(), d.xtype, d.ld, d.P, d.n,
                                      W.data_ptr(), B, bf.g.data_ptr(),
                                      E._work(_lib.query("sglm_xtr_work_bytes", d.P, B, d.n), "cuda").data_ptr(), st)),
        ]:
            if name == "chol":
                bf.H.copy_(H[vs[-1]])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            res[name + "_ms"] = e0.elapsed_time(e1)
        res["chol_info_max"] = int(bf.info.max().item())
    print(json.dumps(res))


if __name__ == "__main__":
    main()

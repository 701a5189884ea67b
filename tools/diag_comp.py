"""Diagnose the complement Gram (development tool): C_all (lag) vs the MFMA Gram of the
all-ones mask, and C_all - C_test vs the train mask's MFMA count Gram."""
import os
import sys
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sabatinilab-glm_amd")]


def main():
    import torch
    from sglm_hip import engine as E, folds, synth
    s = synth.make(N=60_000, m=13, L=6, family="poisson", rho=0.05, seed=5)
    d = E.Design.from_events(s.E, s.shifts, s.L - 1, s.N)
    n, P = d.n, d.P
    np.random.seed(2)
    tr, te = folds.cv_idx_from_bucket_ids(np.asarray(s.trial), num_folds=4)[0]
    masks = [folds.mask_from_idx(tr, n), folds.mask_from_idx(te, n), np.ones(n, np.uint8)]
    prob = E.Problem(d, [s.y], masks)
    st = E._stream()
    nsteps, nt = (n + 31) // 32, (P // 256) * (P // 256 + 1) // 2
    W = prob.M.to(torch.float32)
    H = torch.full((3, P, P), float("nan"), dtype=torch.float32, device="cuda")
    ns = types.SimpleNamespace(W=W, H=H, prob=prob, fit_mask=np.array([0, 1, 2]), wc=None,
                               keep=None)
    E._syrk(d, ns, np.arange(3, dtype=np.int32), nsteps, nt, None, st, exact=True)
    Hl = torch.full((1, P, P), float("nan"), dtype=torch.float32, device="cuda")
    ones = torch.ones((1, d.ld), dtype=torch.float32, device="cuda")
    E._lag_gram(d, types.SimpleNamespace(W=ones, H=Hl, up=None), np.zeros(1, np.int32), st)
    h = H.cpu().numpy()
    hl = Hl[0].cpu().numpy()
    blk = np.kron(np.triu(np.ones((P // 128, P // 128), bool)), np.ones((128, 128), bool))
    p = d.p
    print("P", P, "p", p, "n", n, "row0", d.lag.row0, "smin/smax", d.lag.smin, d.lag.smax)
    for name, a, b in (("lag vs mfma(all)", hl, h[2]), ("all-test vs train", h[2] - h[1], h[0]),
                       ("lag-test vs train", hl - h[1], h[0])):
        diff = np.where(blk, np.abs(a - b), 0)
        i, j = np.unravel_index(np.argmax(diff), diff.shape)
        nbad = int(np.sum(diff > 0.5))
        print(f"{name}: max {diff.max():.3f} at ({i},{j}) a={a[i, j]} b={b[i, j]} bad={nbad}")
        bad = np.argwhere(diff > 0.5)
        if bad.size:
            print("  rows", np.unique(bad[:, 0])[:20], "cols", np.unique(bad[:, 1])[:20])


if __name__ == "__main__":
    main()

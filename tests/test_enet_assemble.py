"""cv_enet_path's result assembly (sglm_hip.enet._assemble, vectorised over every (response,
alpha, split)) against the per-fit loop it replaced -- host logic, no GPU."""
import numpy as np
import pytest


def _loop(w, b, sw, conv, ss, yyh, cnt, c_pm, R, A, K, score_method):
    out = []
    for r in range(R):
        per = []
        for j in range(A):
            p = w.shape[1]
            cv_coefs, cv_b = np.zeros((p, K)), np.zeros(K)
            s_tr, s_te = np.zeros(K), np.zeros(K)
            ss_res = ss_tot = n_te = 0.0
            n_iter, conv_all, refit = [], True, None
            for k in list(range(K)) + [-1]:
                i = (r * A + j) * (K + 1) + (K if k < 0 else k)
                n_iter.append(int(sw[i]))
                conv_all &= bool(conv[i])
                if k < 0:
                    refit = (w[i].copy(), float(b[i]))
                    continue
                cv_coefs[:, k], cv_b[k] = w[i], b[i]
                for side, mt, dst in ((0, 2 * k, s_tr), (1, 2 * k + 1, s_te)):
                    sres = float(ss[i, side])
                    nm = cnt[mt]
                    ym = float(c_pm[r, mt]) / nm if nm else 0.0
                    sst = max(yyh[mt, r] - nm * ym * ym, 0.0)
                    if nm == 0:
                        dst[k] = np.nan
                    elif score_method == "r2":
                        dst[k] = (1.0 if sres == 0 else 0.0) if sst == 0 else 1.0 - sres / sst
                    else:
                        dst[k] = -sres / nm
                    if side == 1:
                        ss_res += sres
                        ss_tot += sst
                        n_te += nm
            per.append({"cv_coefs": cv_coefs, "cv_intercepts": cv_b, "cv_scores_train": s_tr,
                        "cv_scores_test": s_te, "cv_mean_score_train": np.mean(s_tr),
                        "cv_mean_score": np.mean(s_te), "cv_std_score": np.std(s_te),
                        "cv_R2_score": 0 if ss_tot == 0 else 1 - ss_res / ss_tot,
                        "cv_mse_score": ss_res / n_te if n_te else np.nan,
                        "refit_coef": refit[0], "refit_intercept": refit[1],
                        "n_iter": n_iter, "converged": conv_all})
        out.append(per)
    return out


@pytest.mark.parametrize("method", ["r2", "mse"])
def test_assemble_matches_loop(method):
    from sglm_hip.enet import _assemble
    rng = np.random.default_rng(1)
    R, A, K, p = 3, 4, 5, 7
    nf = R * A * (K + 1)
    w, b = rng.normal(size=(nf, p)), rng.normal(size=nf)
    sw = rng.integers(1, 9, nf)
    conv = rng.random(nf) > 0.1
    ss = rng.random((nf, 2)) * 10
    ss[3, 1] = 0.0
    F = 2 * K + 1
    cnt = rng.integers(50, 100, F).astype(float)
    cnt[3] = 0.0                                   # an empty test mask
    yyh = rng.random((F, R)) * 100 + 50
    c_pm = rng.normal(size=(R, F)) * 5
    yyh[1, 0] = cnt[1] * (c_pm[0, 1] / cnt[1]) ** 2   # SS_tot = 0 on one test mask
    got = _assemble(w, b, sw, conv, ss, yyh, cnt, c_pm, R, A, K, method)
    ref = _loop(w, b, sw, conv, ss, yyh, cnt, c_pm, R, A, K, method)
    for r in range(R):
        for j in range(A):
            g, q = got[r][j], ref[r][j]
            assert set(g) == set(q)
            for key in q:
                if isinstance(q[key], np.ndarray):
                    np.testing.assert_allclose(g[key], q[key], rtol=1e-12, atol=1e-12,
                                               equal_nan=True, err_msg=key)
                elif isinstance(q[key], float) and np.isnan(q[key]):
                    assert np.isnan(g[key]), key
                else:
                    assert g[key] == pytest.approx(q[key], rel=1e-12, abs=1e-12), key

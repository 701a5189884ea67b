"""``sglm.models.eval`` (sglm/sglm/models/eval.py)."""
import time

import numpy as np

from sglm.models import sglm


def calc_l1(coeffs):
    return np.sum(np.abs(coeffs))


def calc_l2(coeffs):
    return np.sum(np.square(coeffs))


def print_best_model_info(X_setup, best_score, best_params, best_model, start,
                          show_non_zero_coefs=False):
    """eval.py:12-45."""
    print()
    print('---')
    print()
    if show_non_zero_coefs:
        print('Non-Zero Coeffs:')
        for ic, coef in enumerate(best_model.coef_):
            if np.abs(coef) > 1e-10:
                print(f'> {coef}: {X_setup.columns[ic]}')
    print(f'Best Score: {best_score}')
    print(f'Best Params: {best_params}')
    print(f'Best Model: {best_model}')
    print(f'Best Model — Intercept: {best_model.intercept_}')
    print(f'Overall RunTime: {time.time() - start}')
    print()


def training_fit_holdout_score(X_setup, y_setup, X_holdout, y_holdout, best_params):
    """eval.py:48-69: refit with ``best_params`` (no ``model_name`` in them -> the default
    family, as in the reference) and score on the holdout set."""
    glm = sglm.fit_GLM(X_setup, y_setup, **best_params)
    return glm, glm.r2_score(X_holdout, y_holdout), glm.neg_mse_score(X_holdout, y_holdout)

"""Drop-in for ``backend/sglm_.py`` — the reference keeps a byte-identical copy of sglm.py
under this name and ``sglm_cv`` imports it (backend/sglm_cv.py:3).  Same objects here."""
from sglm import (GLM, ElasticNet, Lasso, LinearRegression, LogisticRegression,  # noqa: F401
                  NotYetImplementedError, PoissonRegressor, Ridge, TweedieRegressor, calc_R2)

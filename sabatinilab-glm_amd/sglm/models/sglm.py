"""``sglm.models.sglm`` (sglm/sglm/models/sglm.py): the same GLM as the backend module —
``GLM``, ``calc_R2``, ``fit_GLM`` and the estimator classes, running on the MI355X engine."""
from sglm import (GLM, ElasticNet, Lasso, LinearRegression, LogisticRegression,  # noqa: F401
                  NotYetImplementedError, PoissonRegressor, Ridge, TweedieRegressor, calc_R2,
                  fit_GLM)

"""``sglm.models.sglm_cv`` (sglm/sglm/models/sglm_cv.py): the CV grid of the backend
(cv_glm_single_params / cv_glm_mult_params / generate_mult_params / SGLM_worker — one batched
MI355X solve per grid) plus the package's ``simple_cv_fit`` (:18-61) and
``cv_idx_by_timeframe`` (:64-87)."""
from sglm_cv import (SGLM_worker, cv_glm_mult_params, cv_glm_single_params,  # noqa: F401
                     generate_mult_params)
from sglm_ez import cv_idx_by_timeframe, simple_cv_fit  # noqa: F401

"""CPU oracle for the sglm hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import anything from this package, and only as the checker / the timed CPU baseline.
The product (``sabatinilab-glm_amd/``) never imports it and has no CPU fallback.

What it restates (float64 numpy, reference citations in each module):

* ``glm_ref``   — the objectives / solvers the reference reaches through
                  ``backend/sglm.py:95-130`` (sklearn 1.7.2 estimators), restated as a
                  float64 damped-Newton solver plus the Gaussian closed forms.
* ``cv_ref``    — ``backend/sglm_cv.py`` aggregation (``cv_glm_single_params``,
                  ``cv_glm_mult_params``, ``generate_mult_params``) and ``calc_R2``.
* ``folds_ref`` — ``backend/sglm_pp.py:218-264`` / ``backend/sglm_ez.py:311-343`` fold
                  generation, i.e. sklearn ``GroupShuffleSplit`` on the global RNG.
* ``pp_ref``    — ``backend/sglm_pp.py`` timeshift family and
                  ``sglm/sglm/features/setup_model_fit.py:43-96``.

Pinning: every function here is checked in ``tests/test_oracle_golden.py`` against the
fixtures in ``tests/golden/`` (sklearn 1.7.2 called directly — never the reference, whose
import was denied, SURVEY.md §8(c) — plus the known answers of
``backend/test/test_sglm_pp.py``).
"""

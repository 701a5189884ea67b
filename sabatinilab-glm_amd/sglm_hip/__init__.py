"""sglm_hip — MI355X-native engine behind the sglm drop-in modules.

Modules: ``_lib`` (ctypes C ABI), ``engine`` (batched IRLS on device), ``folds`` (bit-exact
GroupShuffleSplit), ``timeshift`` (lag-expansion kernel entry), ``estimators`` (the
sklearn-protocol objects GLM instantiates), ``grid`` (batched CV grid), ``synth``.
"""
from . import _lib  # noqa: F401

__all__ = ["_lib"]

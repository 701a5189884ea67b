"""``sglm.features.sglm_pp`` (sglm/sglm/features/sglm_pp.py): the backend preprocessing
module (``sglm_pp``: shift / timeshift / timeshift_multiple on the HIP lag kernel, zscore,
diff, bucket ids, ...) together with the column-level timeshift helpers the package keeps
in this file (features/sglm_pp.py:25-183, the backend has them in sglm_ez)."""
from sglm_pp import *  # noqa: F401,F403
from sglm_pp import (bucket_ids_by_timeframe, concat_all_shifts, concat_pandas_shifts,  # noqa: F401
                     cv_idx_from_bucket_ids, detrend_data, diff, get_column_nums,
                     get_numpy_version, lambda_min_max, min_max_scale, shift, timeshift,
                     timeshift_multiple, zscore)
from sglm_ez import (add_timeshifts_by_sl_to_col_list, add_timeshifts_to_col_list,  # noqa: F401
                     diff_cols, timeshift_cols, timeshift_cols_by_signal_length)

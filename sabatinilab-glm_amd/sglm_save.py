"""Drop-in for ``sglm_save.py`` (sglm_save.py:7-69): the ``GLM_data`` results container that
downstream notebooks pickle and load.  Same module and class name, so files written by the
reference unpickle into this class and vice versa.

Fixed on purpose (API unchanged): ``load`` restores ``self.data`` from the pickled object
(the reference assigns the whole unpickled ``GLM_data`` to ``self.data``, :27-33) — a file
holding a bare dict (as some notebooks write) is accepted too.  Output arrays follow the
reference's formats: ``coef_`` float64 (p,), ``intercept_`` a float (np.save -> shape ())."""
from collections import defaultdict  # noqa: F401  (the reference imports it)
import pickle
from os.path import exists


class GLM_data():
    def __init__(self, file_dir, filename):
        self.file_dir = file_dir
        self.filename = filename
        self.data = {}
        self.data['fit_results'] = []

    def save(self, overwrite=False):
        path_to_file = self.file_dir + '/' + self.filename
        if not exists(path_to_file) or overwrite:
            with open(path_to_file, 'wb') as f:
                pickle.dump(self, f)
            print('SGLM file saved to: ' + path_to_file)
        else:
            print('File already exists. Set overwrite=True to overwrite.')

    def load(self):
        path_to_file = self.file_dir + '/' + self.filename
        if not exists(path_to_file):
            print('File does not exist.')
            return
        with open(path_to_file, 'rb') as f:
            obj = pickle.load(f)
        self.data = obj.data if isinstance(obj, GLM_data) else obj

    def set_uid(self, uid):
        self.data['uid'] = uid

    def set_filename(self, filename):
        self.data['filename'] = filename

    def set_basedata(self, basedata):
        self.data['basedata'] = basedata

    def set_X_cols(self, X_cols):
        self.data['X_cols'] = X_cols

    def set_gss_info(self, folds, pholdout, pgss, gssid=None):
        self.data['gss_info'] = {'folds': folds, 'pholdout': pholdout, 'pgss': pgss,
                                 'gssid': gssid}

    def set_timeshifts(self, negorder, posorder):
        self.data['negorder'] = negorder
        self.data['posorder'] = posorder

    def append_fit_results(self, response_col, hyperparams, glm_model=None, scores=None,
                           dropped_cols=[], gssids=None):
        scores = {} if scores is None else scores
        for score_id in ['tr_witi', 'tr_noiti', 'gss_witi', 'gss_noiti', 'holdout_witi',
                         'holdout_noiti']:
            if score_id not in scores:
                scores[score_id] = None
        self.data['fit_results'].append({'response_col': response_col,
                                         'hyperparams': hyperparams,
                                         'glm_model_gss': glm_model,
                                         'dropped_cols': dropped_cols,
                                         'scores': scores,
                                         'gss_mse': None,
                                         'refit_mse': None,
                                         'gssids': gssids})

"""Drop-in for the reference's models/GateUnits.py: SGU2 / SGU2Model run
inference on the GPU (gate_units.py, sgmm_sgu2_forward) with the reference's
checkpoint format; SGU1 stays the host xgboost regressor it is in the
reference (GateUnits.py:7-40), built lazily so that importing this module does
not need xgboost until an SGU1 is constructed."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from _sgmm_path import sgmm  # noqa: E402
from sgmm_amd import gate_units as _gu  # noqa: E402

SGU2 = _gu.SGU2
SGU2Model = _gu.SGU2Model


class SGU1:
    """The xgboost signal gate unit (host side, GateUnits.py:7-40)."""

    PARAMS = dict(max_depth=4, min_child_weight=4, subsample=1.0, colsample_bytree=1.0, learning_rate=0.01,
                  reg_alpha=0.01, objective="reg:squarederror", n_estimators=1000, early_stopping_rounds=20)

    def __init__(self, model_path=None):
        import xgboost as xgb  # not in this image; the reference imports it at module load
        self.params = dict(self.PARAMS)
        self.model = xgb.XGBRegressor(**self.params)
        self.model_path = model_path

    def train(self, X_train, y_train, X_val, y_val):
        self.model.fit(X_train, y_train, eval_set=[(X_val, y_val)], verbose=False)

    def predict(self, X):
        return self.model.predict(X)

    def save(self, path):
        self.model.save_model(path)

    def load(self, path):
        self.model.load_model(path)

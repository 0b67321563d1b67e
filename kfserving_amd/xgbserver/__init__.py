from .model import XGBoostModel  # noqa: F401
from .xgboost_model_repository import XGBoostModelRepository  # noqa: F401

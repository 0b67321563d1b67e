from .model import LightGBMModel  # noqa: F401
from .lightgbm_model_repository import LightGBMModelRepository  # noqa: F401

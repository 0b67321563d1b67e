from .model import SKLearnModel  # noqa: F401
from .sklearn_model_repository import SKLearnModelRepository  # noqa: F401

"""Model-file loaders producing the canonical :class:`~kfserving_amd.forest.Forest`."""
from .xgboost_format import load_xgboost_model, parse_xgboost_bytes  # noqa: F401
from .lightgbm_format import load_lightgbm_model, parse_lightgbm_text  # noqa: F401
from .sklearn_format import forest_from_sklearn, load_tree_arrays  # noqa: F401

"""Mirror of the python/kfserving model-server API the tree plugins plug into."""
from .errors import HTTPError  # noqa: F401
from .kfmodel import KFModel  # noqa: F401
from .kfmodel_repository import KFModelRepository, MODEL_MOUNT_DIRS  # noqa: F401
from .storage import Storage  # noqa: F401
from . import v2  # noqa: F401
from .kfserver import KFServer  # noqa: F401,E402

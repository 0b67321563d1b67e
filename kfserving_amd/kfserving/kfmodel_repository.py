"""KFModelRepository (mirror of python/kfserving/kfserving/kfmodel_repository.py:21-54)."""
from typing import List, Optional

MODEL_MOUNT_DIRS = "/mnt/models"


class KFModelRepository:
    """Model repository interface, follows NVIDIA Triton's `model-repository` extension."""

    def __init__(self, models_dir: str = MODEL_MOUNT_DIRS):
        self.models = {}
        self.models_dir = models_dir

    def set_models_dir(self, models_dir):  # used for unit tests
        self.models_dir = models_dir

    def get_model(self, name: str):
        return self.models.get(name, None)

    def get_models(self) -> List:
        return list(self.models.values())

    def is_model_ready(self, name: str):
        model = self.get_model(name)
        return False if model is None else model.ready

    def update(self, model) -> None:
        self.models[model.name] = model

    def load(self, name: str) -> bool:
        pass

    def unload(self, name: str):
        if name in self.models:
            del self.models[name]
        else:
            raise KeyError(f"model {name} does not exist")

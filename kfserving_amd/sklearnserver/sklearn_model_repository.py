"""SKLearnModelRepository (mirror of python/sklearnserver/sklearnserver/sklearn_model_repository.py:20-29)."""
import os

from ..kfserving.kfmodel_repository import MODEL_MOUNT_DIRS, KFModelRepository
from .model import SKLearnModel


class SKLearnModelRepository(KFModelRepository):
    def __init__(self, model_dir: str = MODEL_MOUNT_DIRS):
        super().__init__(model_dir)

    async def load(self, name: str) -> bool:
        model = SKLearnModel(name, os.path.join(self.models_dir, name))
        if model.load():
            self.update(model)
        return model.ready

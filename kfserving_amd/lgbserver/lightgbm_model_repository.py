"""LightGBMModelRepository (mirror of python/lgbserver/lgbserver/lightgbm_model_repository.py:20-29)."""
import os

from ..kfserving.kfmodel_repository import MODEL_MOUNT_DIRS, KFModelRepository
from .model import LightGBMModel


class LightGBMModelRepository(KFModelRepository):
    def __init__(self, model_dir: str = MODEL_MOUNT_DIRS, nthread: int = 1):
        super().__init__(model_dir)
        self.nthread = nthread

    async def load(self, name: str) -> bool:
        model = LightGBMModel(name, os.path.join(self.models_dir, name), self.nthread)
        if model.load():
            self.update(model)
        return model.ready

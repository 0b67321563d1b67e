"""python -m kfserving_amd.lgbserver --model_dir D [--model_name M] [--nthread N]
(mirror of python/lgbserver/lgbserver/__main__.py:24-49; workers forced to 1
as in the reference)."""
import argparse
import logging
import sys

from ..kfserving import kfserver
from .lightgbm_model_repository import LightGBMModelRepository
from .model import LightGBMModel

DEFAULT_MODEL_NAME = "default"
DEFAULT_LOCAL_MODEL_DIR = "/tmp/model"
DEFAULT_NTHREAD = 1

parser = argparse.ArgumentParser(parents=[kfserver.parser])
parser.add_argument('--model_dir', required=True,
                    help='A URI pointer to the model directory')
parser.add_argument('--model_name', default=DEFAULT_MODEL_NAME,
                    help='The name that the model is served under.')
parser.add_argument('--nthread', default=DEFAULT_NTHREAD,
                    help='Number of threads to use by LightGBM.')
args, _ = parser.parse_known_args()

if __name__ == "__main__":
    model = LightGBMModel(args.model_name, args.model_dir, args.nthread)
    try:
        model.load()
    except Exception:
        ex_type, ex_value = sys.exc_info()[:2]
        logging.error(f"fail to load model {args.model_name} from dir {args.model_dir}. "
                      f"exception type {ex_type}, exception msg: {ex_value}")
    model_repository = LightGBMModelRepository(args.model_dir, args.nthread)
    kfserver.KFServer(workers=1, registered_models=model_repository) \
        .start([model] if model.ready else [])

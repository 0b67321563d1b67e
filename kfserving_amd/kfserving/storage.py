"""Storage.download -- local-path subset of python/kfserving/kfserving/storage.py:44-80,207-225.

Remote stores (gs://, s3://, azure blob, http) are out of scope for the
tree-predict hot path and raise.
"""
import glob
import logging
import os
import tempfile

from .kfmodel_repository import MODEL_MOUNT_DIRS

_LOCAL_PREFIX = "file://"
_REMOTE_PREFIXES = ("gs://", "s3://", "http://", "https://")


class Storage:
    @staticmethod
    def download(uri: str, out_dir: str = None) -> str:
        logging.info("Copying contents of %s to local", uri)
        is_local = uri.startswith(_LOCAL_PREFIX) or os.path.exists(uri)
        if out_dir is None:
            if is_local:
                return Storage._download_local(uri)
            out_dir = tempfile.mkdtemp()
        elif not os.path.exists(out_dir):
            os.mkdir(out_dir)
        if is_local:
            return Storage._download_local(uri, out_dir)
        if uri.startswith(MODEL_MOUNT_DIRS):
            return out_dir
        if uri.startswith(_REMOTE_PREFIXES) or ".blob.core.windows.net/" in uri:
            raise Exception("Remote storage (%s) is not supported by this build; mount the "
                            "model locally" % uri)
        raise Exception("Cannot recognize storage type for " + uri)

    @staticmethod
    def _download_local(uri, out_dir=None):
        local_path = uri.replace(_LOCAL_PREFIX, "", 1)
        if not os.path.exists(local_path):
            raise RuntimeError("Local path %s does not exist." % (uri))
        if out_dir is None:
            return local_path
        if not os.path.isdir(out_dir):
            os.makedirs(out_dir)
        if os.path.isdir(local_path):
            local_path = os.path.join(local_path, "*")
        for src in glob.glob(local_path):
            _, tail = os.path.split(src)
            dest_path = os.path.join(out_dir, tail)
            logging.info("Linking: %s to %s", src, dest_path)
            os.symlink(src, dest_path)
        return out_dir

"""Checkpoint storage backends (reference: src/neuronx_distributed/trainer/checkpoint_storage.py:28-559).

`FilesysCheckpointStorage` is the production path.  `S3CheckpointStorage` keeps the reference's
interface (multipart upload, exponential back-off on throttling) and is gated on `boto3` being
importable (it is not in this image): constructing it without boto3 raises a clear error.
"""

from __future__ import annotations

import io
import os
import shutil
import time
from typing import Any, List

import torch


class BaseCheckpointStorage:
    def __init__(self, dirname: str):
        self._dirname = dirname

    def dirname(self) -> str:
        return self._dirname

    def is_checkpoint_xser(self, tag: str) -> bool:
        return self.file_exists(os.path.join(tag, "model", "dp_rank_00_tp_rank_00_pp_rank_00.pt.tensors")) or \
            self.dir_exists(os.path.join(tag, "model", "dp_rank_00_tp_rank_00_pp_rank_00.pt.tensors"))

    def list_checkpoint_tags(self) -> List[str]:
        """Tags ordered oldest -> newest (by modification time of their directory)."""
        raise NotImplementedError

    def get_latest_tag(self) -> str:
        """Newest tag whose `done` marker exists."""
        tags = [t for t in self.list_checkpoint_tags() if self.file_exists(os.path.join(t, "done"))]
        if not tags:
            raise RuntimeError(f"no completed checkpoint under {self._dirname}")
        return tags[-1]

    # abstract I/O
    def file_exists(self, filename: str) -> bool: raise NotImplementedError
    def dir_exists(self, dirname: str) -> bool: raise NotImplementedError
    def is_dir(self, path: str) -> bool: raise NotImplementedError
    def find_files(self, ext: str, max_depth: int = -1) -> List[str]: raise NotImplementedError
    def save_text(self, text: str, filename: str) -> None: raise NotImplementedError
    def save_object(self, obj: Any, filename: str) -> None: raise NotImplementedError
    def load_object(self, filename: str, map_location=None, weights_only: bool = True) -> Any: raise NotImplementedError
    def create_dir(self, dirname: str, exist_ok: bool = True) -> None: raise NotImplementedError
    def remove_dir(self, dirname: str) -> None: raise NotImplementedError
    def remove_file(self, filename: str) -> None: raise NotImplementedError


class FilesysCheckpointStorage(BaseCheckpointStorage):
    def _p(self, name: str) -> str:
        return os.path.join(self._dirname, name)

    def list_checkpoint_tags(self) -> List[str]:
        if not os.path.isdir(self._dirname):
            return []
        # only directories carrying the `checkpoint` begin marker are tags: anything else a user
        # keeps under the checkpoint dir (logs, tensorboard, outputs) is never listed, so never GC'd
        tags = [d for d in os.listdir(self._dirname) if os.path.isfile(self._p(os.path.join(d, "checkpoint")))]
        tags.sort(key=lambda d: os.path.getmtime(self._p(os.path.join(d, "checkpoint"))))
        return tags

    def file_exists(self, filename: str) -> bool:
        return os.path.exists(self._p(filename))

    def dir_exists(self, dirname: str) -> bool:
        return os.path.isdir(self._p(dirname))

    def is_dir(self, path: str) -> bool:
        return os.path.isdir(self._p(path))

    def find_files(self, ext: str, max_depth: int = -1) -> List[str]:
        out = []
        for root, _, files in os.walk(self._dirname):
            for f in files:
                if f.endswith(ext):
                    out.append(os.path.relpath(os.path.join(root, f), self._dirname))
        return out

    def save_text(self, text: str, filename: str) -> None:
        os.makedirs(os.path.dirname(self._p(filename)) or self._dirname, exist_ok=True)
        with open(self._p(filename), "w") as f:
            f.write(text)

    def save_object(self, obj: Any, filename: str) -> None:
        path = self._p(filename)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        tmp = f"{path}.tmp.{os.getpid()}"   # unique per writer: concurrent writers never share a tmp
        torch.save(obj, tmp)
        os.replace(tmp, path)

    def load_object(self, filename: str, map_location=None, weights_only: bool = True) -> Any:
        return torch.load(self._p(filename), map_location=map_location, weights_only=weights_only)

    def create_dir(self, dirname: str, exist_ok: bool = True) -> None:
        os.makedirs(self._p(dirname), exist_ok=exist_ok)

    def remove_dir(self, dirname: str) -> None:
        shutil.rmtree(self._p(dirname), ignore_errors=True)

    def remove_file(self, filename: str) -> None:
        if os.path.exists(self._p(filename)):
            os.remove(self._p(filename))


class S3CheckpointStorage(BaseCheckpointStorage):
    """s3://bucket/prefix storage with retry + exponential back-off (needs boto3)."""

    MAX_RETRY = 8

    def __init__(self, dirname: str):
        super().__init__(dirname)
        try:
            import boto3  # noqa: F401
        except ImportError as e:
            raise RuntimeError("S3 checkpoint storage requires boto3, which is not installed") from e
        import boto3

        assert dirname.startswith("s3://")
        rest = dirname[len("s3://"):]
        self.bucket, _, self.prefix = rest.partition("/")
        self.client = boto3.client("s3")

    def _key(self, name):
        return f"{self.prefix.rstrip('/')}/{name}" if self.prefix else name

    def _retry(self, fn, *a, **kw):
        delay = 1.0
        for attempt in range(self.MAX_RETRY):
            try:
                return fn(*a, **kw)
            except Exception as e:  # pragma: no cover - network
                if "SlowDown" not in str(e) and "Throttl" not in str(e) or attempt == self.MAX_RETRY - 1:
                    raise
                time.sleep(delay)
                delay *= 2

    def list_checkpoint_tags(self) -> List[str]:  # pragma: no cover - network
        resp = self._retry(self.client.list_objects_v2, Bucket=self.bucket, Prefix=self._key(""), Delimiter="/")
        tags = []
        for p in resp.get("CommonPrefixes", []):
            tag = p["Prefix"].rstrip("/").split("/")[-1]
            try:
                head = self._retry(self.client.head_object, Bucket=self.bucket, Key=self._key(f"{tag}/checkpoint"))
            except Exception:
                continue   # no begin marker: not a checkpoint tag
            tags.append((head["LastModified"], tag))
        return [t for _, t in sorted(tags)]

    def file_exists(self, filename: str) -> bool:  # pragma: no cover - network
        try:
            self._retry(self.client.head_object, Bucket=self.bucket, Key=self._key(filename))
            return True
        except Exception:
            return False

    dir_exists = file_exists
    is_dir = file_exists

    def save_text(self, text: str, filename: str) -> None:  # pragma: no cover - network
        self._retry(self.client.put_object, Bucket=self.bucket, Key=self._key(filename), Body=text.encode())

    def save_object(self, obj: Any, filename: str) -> None:  # pragma: no cover - network
        buf = io.BytesIO()
        torch.save(obj, buf)
        self._retry(self.client.upload_fileobj, io.BytesIO(buf.getvalue()), self.bucket, self._key(filename))

    def load_object(self, filename: str, map_location=None, weights_only: bool = True) -> Any:  # pragma: no cover
        buf = io.BytesIO()
        self._retry(self.client.download_fileobj, self.bucket, self._key(filename), buf)
        buf.seek(0)
        return torch.load(buf, map_location=map_location, weights_only=weights_only)

    def create_dir(self, dirname: str, exist_ok: bool = True) -> None:
        return None

    def remove_dir(self, dirname: str) -> None:  # pragma: no cover - network
        resp = self._retry(self.client.list_objects_v2, Bucket=self.bucket, Prefix=self._key(dirname))
        for o in resp.get("Contents", []):
            self._retry(self.client.delete_object, Bucket=self.bucket, Key=o["Key"])

    def remove_file(self, filename: str) -> None:  # pragma: no cover - network
        self._retry(self.client.delete_object, Bucket=self.bucket, Key=self._key(filename))


def create_checkpoint_storage(dirname: str) -> BaseCheckpointStorage:
    if dirname.startswith("s3://"):
        return S3CheckpointStorage(dirname)
    return FilesysCheckpointStorage(dirname)

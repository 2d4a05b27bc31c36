"""Advisory file locks for the per-model single-writer rule.

The reference shares one append-mode ``result.txt`` and one PS/worker container pair
between every launch, serialised only by ``pkill -9 python`` before each start
(apps/construction/views.py:128-129; construct_distribute.py:409).  Here two locks
replace that:

* ``model_dir/.submit.lock`` — held (blocking) while the job manager checks for an
  active job of the model and inserts a new one, so two API workers cannot both admit
  a job for the same (user, model);
* ``model_dir/.writer.lock`` — held (non-blocking try) by the process that writes the
  model dir's ``result.txt`` / ``metrics.jsonl`` / checkpoints for the job's whole run;
  a second writer fails fast instead of interleaving lines.  The kernel drops the lock
  when the holder dies, so a crashed job never leaves a stale lock behind.

``flock`` locks belong to the open file description: two opens in ONE process (two
packed jobs in a GPU host) still exclude each other.
"""
from __future__ import annotations

import contextlib
import fcntl
import os
from typing import Iterator, Optional

SUBMIT_LOCK = ".submit.lock"
WRITER_LOCK = ".writer.lock"


class LockHeld(RuntimeError):
    """The lock is held by another writer."""


@contextlib.contextmanager
def locked(path: str) -> Iterator[None]:
    """Exclusive blocking lock on ``path`` (created if missing) for the ``with`` body."""
    fd = os.open(path, os.O_RDWR | os.O_CREAT, 0o644)
    try:
        fcntl.flock(fd, fcntl.LOCK_EX)
        yield
    finally:
        try:
            fcntl.flock(fd, fcntl.LOCK_UN)
        finally:
            os.close(fd)


class WriterLock:
    """Non-blocking exclusive lock held for a job's lifetime (``release`` is idempotent)."""

    def __init__(self, model_dir: str):
        self.path = os.path.join(model_dir, WRITER_LOCK)
        self.fd: Optional[int] = os.open(self.path, os.O_RDWR | os.O_CREAT, 0o644)
        try:
            fcntl.flock(self.fd, fcntl.LOCK_EX | fcntl.LOCK_NB)
        except OSError:
            holder = ""
            try:
                holder = os.pread(self.fd, 64, 0).decode(errors="replace").strip()
            except OSError:
                pass
            os.close(self.fd)
            self.fd = None
            raise LockHeld(f"another job is writing {model_dir} (pid {holder or '?'})") from None
        os.ftruncate(self.fd, 0)
        os.pwrite(self.fd, str(os.getpid()).encode(), 0)

    def release(self) -> None:
        if self.fd is None:
            return
        try:
            fcntl.flock(self.fd, fcntl.LOCK_UN)
        finally:
            os.close(self.fd)
            self.fd = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.release()
        except Exception:
            pass

"""Settings: one env-driven object replacing the reference's config layers.

Reference: Django settings.py (hard-coded SECRET_KEY, MySQL and SMTP credentials,
DEBUG=True, ALLOWED_HOSTS='*'; settings.py:22-170) and module constants in
global_settings.py (storage root, container IDs, PS/worker host:port).  None of those
secrets are reproduced: everything comes from ``CSA_*`` environment variables with safe
local defaults.

| variable              | default                         | meaning                               |
|-----------------------|---------------------------------|---------------------------------------|
| CSA_STORAGE_ROOT      | ~/.cloud_server_amd             | workspace root (replaces /root/)      |
| CSA_DB_PATH           | <root>/server.sqlite3           | SQLite database file                  |
| CSA_GPUS              | all visible                     | comma list of GPU ids the scheduler uses |
| CSA_EXECUTOR          | process                         | process / thread / inline job runner  |
| CSA_TOKEN_TTL_S       | 0 (never expires)               | auth token lifetime                   |
| CSA_ALLOW_URL_FETCH   | 1                               | allow the ``url`` dataset type (http/https only) |
| CSA_URL_ALLOW_PRIVATE | 0                               | let URL datasets reach loopback/private hosts |
| CSA_MAX_UPLOAD_MB     | 512                             | request body limit                    |
| CSA_CORS_ORIGINS      | (none)                          | comma list of allowed CORS origins ("*" = any) |
| CSA_HEARTBEAT_S       | 900                             | a running job silent this long is killed + failed |
| CSA_ENABLE_DEMO       | 0                               | mount the demo "bills" routes (off, as in the reference) |
| CSA_INFER_DEVICE      | auto (the last GPU when one exists) | device of the inference service (HIP forward) and GPU preprocessing |
| CSA_SERVE_SLOTS       | 1                               | scheduler slots reserved on the serving GPU for the API process |
| CSA_PACK_JOBS         | 1                               | single-GPU jobs on one GPU share a packed host process |
| CSA_SLOTS_PER_GPU     | 4 packed / 1 unpacked           | concurrent jobs per GPU (profiles/r2_multitenant.md) |
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import List, Optional


def _env(name: str, default: str) -> str:
    return os.environ.get(name, default)


@dataclass
class Settings:
    storage_root: str = field(default_factory=lambda: os.path.abspath(os.path.expanduser(
        _env("CSA_STORAGE_ROOT", "~/.cloud_server_amd"))))
    db_path: str = ""
    gpus: Optional[List[int]] = None
    executor: str = field(default_factory=lambda: _env("CSA_EXECUTOR", "process"))
    token_ttl_s: int = field(default_factory=lambda: int(_env("CSA_TOKEN_TTL_S", "0")))
    allow_url_fetch: bool = field(default_factory=lambda: _env("CSA_ALLOW_URL_FETCH", "1") == "1")
    url_allow_private: bool = field(default_factory=lambda: _env("CSA_URL_ALLOW_PRIVATE", "0") == "1")
    max_upload_mb: int = field(default_factory=lambda: int(_env("CSA_MAX_UPLOAD_MB", "512")))
    preprocess_backend: str = field(default_factory=lambda: _env("CSA_PREPROCESS_BACKEND", "auto"))
    train_backend: str = field(default_factory=lambda: _env("CSA_TRAIN_BACKEND", "auto"))
    cors_origins: List[str] = field(default_factory=lambda: [o.strip() for o in _env("CSA_CORS_ORIGINS", "").split(",")
                                                             if o.strip()])
    heartbeat_s: float = field(default_factory=lambda: float(_env("CSA_HEARTBEAT_S", "900")))
    enable_demo: bool = field(default_factory=lambda: _env("CSA_ENABLE_DEMO", "0") == "1")
    # measured on one MI355X (bench.py --jobs K): K jobs packed as branches of one graph
    # give 1.44x / 1.92x / 2.07x aggregate at K = 2 / 4 / 8, K separate processes give
    # 0.75x / 0.68x / 0.69x — so pack, 4 per GPU (8 adds 8% for 2x per-job latency), and
    # without packing run one job per GPU at a time
    infer_device: str = field(default_factory=lambda: _env("CSA_INFER_DEVICE", "auto"))
    pack_jobs: bool = field(default_factory=lambda: _env("CSA_PACK_JOBS", "1") == "1")
    slots_per_gpu: int = field(default_factory=lambda: int(_env("CSA_SLOTS_PER_GPU", "0")))
    serve_slots: int = field(default_factory=lambda: int(_env("CSA_SERVE_SLOTS", "1")))

    def __post_init__(self):
        if not self.db_path:
            self.db_path = _env("CSA_DB_PATH", os.path.join(self.storage_root, "server.sqlite3"))
        if self.gpus is None:
            g = _env("CSA_GPUS", "")
            self.gpus = [int(x) for x in g.split(",") if x.strip()] if g else None
        if self.slots_per_gpu <= 0:
            self.slots_per_gpu = 4 if self.pack_jobs else 1
        os.makedirs(self.storage_root, exist_ok=True)

    # ---- workspace layout, per user and model; no global scratch ----
    def user_root(self, uid: int) -> str:
        return os.path.join(self.storage_root, "NJUCloud", str(uid))

    def data_dir(self, uid: int, file_class: str) -> str:
        return os.path.join(self.user_root(uid), "data", file_class)

    def model_dir(self, uid: int, model: str) -> str:
        return os.path.join(self.user_root(uid), "model", model)


_SETTINGS: Optional[Settings] = None


def get_settings() -> Settings:
    global _SETTINGS
    if _SETTINGS is None:
        _SETTINGS = Settings()
    return _SETTINGS


def set_settings(s: Settings) -> None:
    global _SETTINGS
    _SETTINGS = s

"""Persistence: SQLite (stdlib) in place of the reference's MySQL + Django ORM.

Tables mirror the reference models plus what the framework-provided apps stored:

* ``users``      — django.contrib.auth User (C05): username, email, password hash, names
* ``tokens``     — rest_framework.authtoken Token (one key per user)
* ``raw_data``   — apps/data/models.py:6-32 ``RawData``: created_at, file_path (relative to
  the storage root), file_type in {doc, audio, picture, code}, owner
* ``jobs``       — NEW: training jobs (the reference had no job record; the only state
  was result.txt inside a container)
* ``reset_tokens`` / ``email_keys`` — password reset and e-mail verification keys

Passwords: PBKDF2-HMAC-SHA256 with a per-user salt (Django's default hasher family).
One connection per thread; every write is a short transaction.
"""
from __future__ import annotations

import hashlib
import hmac
import json
import os
import secrets
import sqlite3
import threading
import time
from typing import Any, Dict, List, Optional, Tuple

SCHEMA = """
CREATE TABLE IF NOT EXISTS users (
  id INTEGER PRIMARY KEY AUTOINCREMENT,
  username TEXT UNIQUE NOT NULL,
  email TEXT NOT NULL DEFAULT '',
  password TEXT NOT NULL,
  first_name TEXT NOT NULL DEFAULT '',
  last_name TEXT NOT NULL DEFAULT '',
  is_staff INTEGER NOT NULL DEFAULT 0,
  email_verified INTEGER NOT NULL DEFAULT 0,
  date_joined REAL NOT NULL
);
CREATE TABLE IF NOT EXISTS tokens (
  key TEXT PRIMARY KEY,
  user_id INTEGER UNIQUE NOT NULL REFERENCES users(id) ON DELETE CASCADE,
  created REAL NOT NULL
);
CREATE TABLE IF NOT EXISTS raw_data (
  id INTEGER PRIMARY KEY AUTOINCREMENT,
  created_at REAL NOT NULL,
  file_path TEXT NOT NULL,
  file_type TEXT NOT NULL DEFAULT 'doc',
  owner_id INTEGER NOT NULL REFERENCES users(id) ON DELETE CASCADE
);
CREATE TABLE IF NOT EXISTS jobs (
  id INTEGER PRIMARY KEY AUTOINCREMENT,
  owner_id INTEGER NOT NULL REFERENCES users(id) ON DELETE CASCADE,
  model TEXT NOT NULL,
  datatype TEXT NOT NULL,
  config TEXT NOT NULL,
  state TEXT NOT NULL,
  created REAL NOT NULL,
  started REAL,
  finished REAL,
  gpu TEXT,
  error TEXT
);
CREATE TABLE IF NOT EXISTS reset_tokens (
  token TEXT PRIMARY KEY,
  user_id INTEGER NOT NULL REFERENCES users(id) ON DELETE CASCADE,
  created REAL NOT NULL
);
CREATE TABLE IF NOT EXISTS email_keys (
  key TEXT PRIMARY KEY,
  user_id INTEGER NOT NULL REFERENCES users(id) ON DELETE CASCADE,
  created REAL NOT NULL
);
CREATE TABLE IF NOT EXISTS bills (
  id INTEGER PRIMARY KEY AUTOINCREMENT,
  created REAL NOT NULL,
  goods TEXT NOT NULL,
  price REAL NOT NULL,
  amount INTEGER NOT NULL DEFAULT 1,
  description TEXT NOT NULL DEFAULT 'no description',
  owner_id INTEGER NOT NULL REFERENCES users(id) ON DELETE CASCADE
);
CREATE INDEX IF NOT EXISTS raw_data_owner ON raw_data(owner_id, created_at);
CREATE INDEX IF NOT EXISTS jobs_owner ON jobs(owner_id, model);
"""

FILE_TYPES = ("doc", "audio", "picture", "code")   # RawData.FILE_TYPE_CHOICES (models.py:8-17)
PBKDF2_ITERS = int(os.environ.get("CSA_PBKDF2_ITERS", "120000"))


def hash_password(pw: str, salt: Optional[str] = None, iters: int = PBKDF2_ITERS) -> str:
    salt = salt or secrets.token_hex(12)
    dk = hashlib.pbkdf2_hmac("sha256", pw.encode(), salt.encode(), iters)
    return f"pbkdf2_sha256${iters}${salt}${dk.hex()}"


def check_password(pw: str, encoded: str) -> bool:
    try:
        algo, iters, salt, h = encoded.split("$")
    except ValueError:
        return False
    dk = hashlib.pbkdf2_hmac("sha256", pw.encode(), salt.encode(), int(iters))
    return hmac.compare_digest(dk.hex(), h)


class Database:
    def __init__(self, path: str):
        self.path = path
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        self._local = threading.local()
        self.conn().executescript(SCHEMA)      # executescript manages its own transaction

    def conn(self) -> sqlite3.Connection:
        c = getattr(self._local, "c", None)
        if c is None:
            c = sqlite3.connect(self.path, timeout=30, isolation_level=None, check_same_thread=False)
            c.row_factory = sqlite3.Row
            c.execute("PRAGMA foreign_keys = ON")
            c.execute("PRAGMA journal_mode = WAL")
            self._local.c = c
        return c

    class _Tx:
        def __init__(self, c):
            self.c = c

        def __enter__(self):
            self.c.execute("BEGIN IMMEDIATE")
            return self.c

        def __exit__(self, et, ev, tb):
            self.c.execute("COMMIT" if et is None else "ROLLBACK")

    def tx(self):
        return self._Tx(self.conn())

    def table_counts(self) -> List[Tuple[str, int]]:
        """(table, row count) of every platform table (the read-only admin index)."""
        c = self.conn()
        names = [r[0] for r in c.execute(
            "SELECT name FROM sqlite_master WHERE type='table' AND name NOT LIKE 'sqlite_%' ORDER BY name")]
        return [(n, int(c.execute(f'SELECT COUNT(*) FROM "{n}"').fetchone()[0])) for n in names]

    # ------------------------------------------------------------------ users
    def create_user(self, username: str, password: str, email: str = "", is_staff: bool = False) -> int:
        with self.tx() as c:
            cur = c.execute(
                "INSERT INTO users(username, email, password, is_staff, date_joined) VALUES (?,?,?,?,?)",
                (username, email, hash_password(password), int(is_staff), time.time()))
            return int(cur.lastrowid)

    def get_user(self, uid: int) -> Optional[Dict[str, Any]]:
        r = self.conn().execute("SELECT * FROM users WHERE id=?", (uid,)).fetchone()
        return dict(r) if r else None

    def find_user(self, username: Optional[str] = None, email: Optional[str] = None) -> Optional[Dict[str, Any]]:
        if username:
            r = self.conn().execute("SELECT * FROM users WHERE username=?", (username,)).fetchone()
        elif email:
            r = self.conn().execute("SELECT * FROM users WHERE lower(email)=lower(?)", (email,)).fetchone()
        else:
            r = None
        return dict(r) if r else None

    def update_user(self, uid: int, **fields) -> None:
        allowed = {k: v for k, v in fields.items()
                   if k in ("username", "email", "first_name", "last_name", "email_verified")}
        if not allowed:
            return
        cols = ", ".join(f"{k}=?" for k in allowed)
        with self.tx() as c:
            c.execute(f"UPDATE users SET {cols} WHERE id=?", (*allowed.values(), uid))

    def set_password(self, uid: int, password: str) -> None:
        """New password hash; every API token / browser session and every outstanding
        reset link of the user is revoked with it (Django invalidates sessions and reset
        tokens once the password hash changes)."""
        with self.tx() as c:
            c.execute("UPDATE users SET password=? WHERE id=?", (hash_password(password), uid))
            c.execute("DELETE FROM tokens WHERE user_id=?", (uid,))
            c.execute("DELETE FROM reset_tokens WHERE user_id=?", (uid,))

    # ------------------------------------------------------------------ tokens
    def token_for(self, uid: int) -> str:
        r = self.conn().execute("SELECT key FROM tokens WHERE user_id=?", (uid,)).fetchone()
        if r:
            return r["key"]
        key = secrets.token_hex(20)       # DRF Token: 40 hex chars
        with self.tx() as c:
            c.execute("INSERT INTO tokens(key, user_id, created) VALUES (?,?,?)", (key, uid, time.time()))
        return key

    def user_for_token(self, key: str, ttl_s: int = 0) -> Optional[Dict[str, Any]]:
        r = self.conn().execute(
            "SELECT u.*, t.created AS token_created FROM tokens t JOIN users u ON u.id=t.user_id WHERE t.key=?",
            (key,)).fetchone()
        if not r:
            return None
        if ttl_s and time.time() - r["token_created"] > ttl_s:
            return None
        return dict(r)

    def delete_token(self, uid: int) -> None:
        with self.tx() as c:
            c.execute("DELETE FROM tokens WHERE user_id=?", (uid,))

    def new_reset_token(self, uid: int) -> str:
        tok = secrets.token_urlsafe(24)
        with self.tx() as c:
            c.execute("INSERT INTO reset_tokens(token, user_id, created) VALUES (?,?,?)", (tok, uid, time.time()))
        return tok

    def use_reset_token(self, uid: int, tok: str, max_age_s: int = 3 * 86400) -> bool:
        r = self.conn().execute("SELECT * FROM reset_tokens WHERE token=? AND user_id=?", (tok, uid)).fetchone()
        if not r or time.time() - r["created"] > max_age_s:
            return False
        with self.tx() as c:
            c.execute("DELETE FROM reset_tokens WHERE token=?", (tok,))
        return True

    def new_email_key(self, uid: int) -> str:
        key = secrets.token_urlsafe(24)
        with self.tx() as c:
            c.execute("INSERT INTO email_keys(key, user_id, created) VALUES (?,?,?)", (key, uid, time.time()))
        return key

    def verify_email_key(self, key: str) -> Optional[int]:
        r = self.conn().execute("SELECT user_id FROM email_keys WHERE key=?", (key,)).fetchone()
        if not r:
            return None
        with self.tx() as c:
            c.execute("DELETE FROM email_keys WHERE key=?", (key,))
            c.execute("UPDATE users SET email_verified=1 WHERE id=?", (r["user_id"],))
        return int(r["user_id"])

    # ------------------------------------------------------------------ raw data
    def add_raw_data(self, owner: int, file_path: str, file_type: str) -> int:
        with self.tx() as c:
            cur = c.execute("INSERT INTO raw_data(created_at, file_path, file_type, owner_id) VALUES (?,?,?,?)",
                            (time.time(), file_path, file_type, owner))
            return int(cur.lastrowid)

    def get_raw_data(self, pk: int) -> Optional[Dict[str, Any]]:
        r = self.conn().execute("SELECT * FROM raw_data WHERE id=?", (pk,)).fetchone()
        return dict(r) if r else None

    def list_raw_data(self, owner: int) -> List[Dict[str, Any]]:
        rows = self.conn().execute("SELECT * FROM raw_data WHERE owner_id=? ORDER BY created_at, id",
                                   (owner,)).fetchall()
        return [dict(r) for r in rows]

    def delete_raw_data(self, pk: int) -> bool:
        with self.tx() as c:
            return c.execute("DELETE FROM raw_data WHERE id=?", (pk,)).rowcount > 0

    # ------------------------------------------------------------------ jobs
    def add_job(self, owner: int, model: str, datatype: str, config: Dict[str, Any]) -> int:
        with self.tx() as c:
            cur = c.execute(
                "INSERT INTO jobs(owner_id, model, datatype, config, state, created) VALUES (?,?,?,?,?,?)",
                (owner, model, datatype, json.dumps(config), "queued", time.time()))
            return int(cur.lastrowid)

    def update_job(self, jid: int, **fields) -> None:
        allowed = {k: v for k, v in fields.items() if k in ("state", "started", "finished", "gpu", "error")}
        if not allowed:
            return
        cols = ", ".join(f"{k}=?" for k in allowed)
        with self.tx() as c:
            c.execute(f"UPDATE jobs SET {cols} WHERE id=?", (*allowed.values(), jid))

    def get_job(self, jid: int) -> Optional[Dict[str, Any]]:
        r = self.conn().execute("SELECT * FROM jobs WHERE id=?", (jid,)).fetchone()
        return dict(r) if r else None

    def jobs_for(self, owner: int, model: Optional[str] = None) -> List[Dict[str, Any]]:
        if model is None:
            rows = self.conn().execute("SELECT * FROM jobs WHERE owner_id=? ORDER BY id", (owner,)).fetchall()
        else:
            rows = self.conn().execute("SELECT * FROM jobs WHERE owner_id=? AND model=? ORDER BY id",
                                       (owner, model)).fetchall()
        return [dict(r) for r in rows]

    def active_jobs(self) -> List[Dict[str, Any]]:
        rows = self.conn().execute(
            "SELECT * FROM jobs WHERE state IN ('queued','running','paused') ORDER BY id").fetchall()
        return [dict(r) for r in rows]

    # ------------------------------------------------------------------ demo bills
    # (demo/models.py:6-28 — the reference's scaffolding example, kept for parity)
    def add_bill(self, owner: int, goods: str, price: float, amount: int = 1,
                 description: str = "no description") -> int:
        with self.tx() as c:
            cur = c.execute("INSERT INTO bills(created, goods, price, amount, description, owner_id) "
                            "VALUES (?,?,?,?,?,?)", (time.time(), goods, price, amount, description, owner))
            return int(cur.lastrowid)

    def _bill_rows(self, where: str = "", args=()) -> List[Dict[str, Any]]:
        rows = self.conn().execute(
            "SELECT b.*, u.username AS owner FROM bills b JOIN users u ON u.id = b.owner_id "
            f"{where} ORDER BY b.created, b.owner_id", args).fetchall()
        return [dict(r) for r in rows]

    def list_bills(self, goods_contains: Optional[str] = None) -> List[Dict[str, Any]]:
        if goods_contains is None:
            return self._bill_rows()
        return self._bill_rows("WHERE b.goods LIKE ? ESCAPE '\\'",
                               ("%" + goods_contains.replace("\\", "\\\\").replace("%", "\\%")
                                .replace("_", "\\_") + "%",))

    def get_bill(self, pk: int) -> Optional[Dict[str, Any]]:
        r = self._bill_rows("WHERE b.id=?", (pk,))
        return r[0] if r else None

    def update_bill(self, pk: int, **fields) -> None:
        allowed = {k: v for k, v in fields.items() if k in ("goods", "price", "amount", "description")}
        if allowed:
            cols = ", ".join(f"{k}=?" for k in allowed)
            with self.tx() as c:
                c.execute(f"UPDATE bills SET {cols} WHERE id=?", (*allowed.values(), pk))

    def delete_bill(self, pk: int) -> bool:
        with self.tx() as c:
            return c.execute("DELETE FROM bills WHERE id=?", (pk,)).rowcount > 0

"""REST API (FastAPI) — the reference's Django REST Framework surface, same paths/payloads.

Route table (reference views in parentheses):

  user     POST /rest-auth/login/ | logout/ | password/reset/ | password/reset/confirm/ |
           password/change/ ; GET/PUT/PATCH /rest-auth/user/ ; POST /rest-auth/registration/
           | registration/verify-email/                     (django-rest-auth, urls.py:27-30)
  data     POST /data/create/ (ModelCreation)  POST /data/tag/ (TagUpload)
           GET|POST /data/list/ (DataView)  GET|DELETE /data/<pk>/ (DataDetail)
  prep     POST|GET /preprocess/ (PreprocessView)  GET /preprocess/operations/list/
  build    POST /construct/options/ (ConfigOptions)  GET /construct/config/ (ConfigView)
           GET /construct/detail/<m>/ (ConfigDetail)
           POST /construct/construction/<m>/<datatype>/ (ConstructView)
           POST /construct/inference/<m>/ (InferenceView)
  runtime  GET /runtime/train/<m>/<iter>/ (TensorResultView)  GET /runtime/kubernetes/
  browser  /login/ /logout/ /password_change/(done/) /password_reset/(done/)
           /reset/<uid>/<token>/ /reset/done/ (django.contrib.auth.urls), /admin/ (api/html_auth.py)
  documented-only in API.md, implemented here: /generation/options/list|next,
           /generation/generate, /generation/run/basic|details|runtime|stop|pause,
           /generation/restore/<job>/, /models/, /models/<m>/, /models/compare/

Auth: ``Authorization: Token <key>`` (rest_framework.authtoken), HTTP Basic, or the
``sessionid`` cookie set by the HTML ``/login/`` form (SessionAuthentication).  Unlike
the reference, every data/model route requires authentication and checks ownership
(quirk 8: DELETE /data/<pk>/ had no owner check; "auth only" routes let anonymous users
write into NJUCloud/None/), names are validated and ``relative_path`` cannot escape the
dataset directory; no shell commands are built from request data.
"""
from __future__ import annotations

import base64
import contextlib
import hmac
import io
import json
import mimetypes
import os
import shutil
import time
import zipfile
from typing import Any, Dict, List, Optional

import torch
from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, Response
from starlette.concurrency import run_in_threadpool

from . import html_auth
from ..config import Settings, get_settings
from ..models.dsl import ConfigError, parse_train_config, spec_to_dict
from ..models.options import CATALOG, get_options
from ..preprocess import ops_ref, pipeline
from ..runtime.devices import node_status
from ..runtime.jobs import JobConflict, JobManager
from ..runtime.trainer import METRICS, RESULT, STATUS, read_train_results
from ..serve.inference import FAIL_NO_MODEL, InferenceService
from ..store.db import FILE_TYPES, Database, check_password
from ..utils import net
from ..utils.files import csv_to_json, dir_tree, safe_join, timestamped_name, valid_name
from .forms import FormError, read_form

COMMON_PASSWORDS = {"password", "12345678", "123456789", "qwertyui", "password1", "iloveyou", "11111111",
                    "abcdefgh", "00000000", "88888888", "1234567890", "qwerty123", "admin123"}


def J(data: Any, status: int = 200) -> JSONResponse:
    return JSONResponse(data, status_code=status)


def _err(detail: str, status: int) -> JSONResponse:
    return J({"detail": detail}, status)


def validate_password(pw: str, username: str = "", email: str = "") -> List[str]:
    """settings.py:123-136 validators: similarity, min length 8, common, numeric."""
    errs = []
    if len(pw) < 8:
        errs.append("This password is too short. It must contain at least 8 characters.")
    if pw.isdigit():
        errs.append("This password is entirely numeric.")
    if pw.lower() in COMMON_PASSWORDS:
        errs.append("This password is too common.")
    for attr in (username, email.split("@")[0] if email else ""):
        if attr and len(attr) >= 3 and (attr.lower() in pw.lower() or pw.lower() in attr.lower()):
            errs.append("The password is too similar to the username.")
            break
    return errs


def create_app(settings: Optional[Settings] = None, executor: Optional[str] = None,
               ngpu: Optional[int] = None, inference_device: Optional[str] = None) -> FastAPI:
    settings = settings or get_settings()
    db = Database(settings.db_path)
    jobs = JobManager(settings, db, executor=executor, ngpu=ngpu)
    dev = inference_device or getattr(settings, "infer_device", "auto")
    if dev == "auto":
        # the serving GPU: the last one (device_count() does not initialise HIP on this
        # image); its scheduler slot is reserved below so packed training avoids it first
        try:
            n = torch.cuda.device_count()
        except Exception:
            n = 0
        dev = f"cuda:{max(min(n, jobs.ngpu) - 1, 0)}" if n > 0 and jobs.ngpu > 0 else "cpu"
    serve_dev = torch.device(dev)
    if serve_dev.type == "cuda":
        serve_dev = torch.device("cuda", serve_dev.index or 0)
        jobs.reserve_serving(serve_dev.index)
    infer = InferenceService(device=str(serve_dev))

    def on_serve_device(fn, *a, **kw):
        """Run ``fn`` with the serving GPU current (GPU preprocessing opens no context on
        another device of the API process)."""
        if serve_dev.type != "cuda":
            return fn(*a, **kw)
        with torch.cuda.device(serve_dev):
            return fn(*a, **kw)

    @contextlib.asynccontextmanager
    async def lifespan(_app):
        yield
        jobs.shutdown()
        infer.close()

    app = FastAPI(title="cloud_server_amd", version="1.0", lifespan=lifespan)
    app.state.settings, app.state.db, app.state.jobs, app.state.infer = settings, db, jobs, infer
    max_bytes = settings.max_upload_mb << 20
    if settings.cors_origins:
        # settings.py:53-82: corsheaders with GET/POST/PUT/PATCH/DELETE/OPTIONS and the
        # x-requested-with/content-type/accept/origin/authorization/x-csrftoken headers
        from fastapi.middleware.cors import CORSMiddleware
        app.add_middleware(CORSMiddleware, allow_origins=settings.cors_origins,
                           allow_methods=["GET", "POST", "PUT", "PATCH", "DELETE", "OPTIONS"],
                           allow_headers=["x-requested-with", "content-type", "accept", "origin",
                                          "authorization", "x-csrftoken"])
    _install_metrics(app, db)

    # ------------------------------------------------------------------ auth helpers
    def current_user(request: Request, csrf_verified: bool = False) -> Optional[Dict[str, Any]]:
        """Token / Basic / session-cookie auth.  ``csrf_verified``: the caller (an HTML
        form handler) already checked the form's CSRF field."""
        h = request.headers.get("authorization", "")
        if h.lower().startswith("token "):
            return db.user_for_token(h.split(None, 1)[1].strip(), settings.token_ttl_s)
        if h.lower().startswith("basic "):
            try:
                u, _, p = base64.b64decode(h.split(None, 1)[1]).decode().partition(":")
            except Exception:
                return None
            user = db.find_user(username=u)
            if user and check_password(p, user["password"]):
                return user
        sid = request.cookies.get(html_auth.COOKIE)     # browser session from /login/
        if sid:
            # SessionAuthentication semantics: a cookie-authenticated unsafe request must
            # carry the CSRF token (double submit: X-CSRFToken header == csrftoken cookie)
            if not csrf_verified and request.method not in ("GET", "HEAD", "OPTIONS", "TRACE"):
                cookie = request.cookies.get(html_auth.CSRF_COOKIE, "")
                header = request.headers.get("x-csrftoken", "")
                if not cookie or not hmac.compare_digest(cookie, header):
                    return None
            return db.user_for_token(sid, settings.token_ttl_s)
        return None

    def need_user(request: Request):
        u = current_user(request)
        if u is None:
            return None, _err("Authentication credentials were not provided.", 401)
        return u, None

    async def form(request: Request):
        try:
            return (*await read_form(request, max_bytes), None)
        except FormError as e:
            return {}, {}, J({"message": "error", "detail": str(e)}, 400)

    def user_json(u: Dict[str, Any]) -> Dict[str, Any]:
        return {"pk": u["id"], "username": u["username"], "email": u["email"],
                "first_name": u["first_name"], "last_name": u["last_name"]}

    def outbox(to: str, subject: str, body: str) -> None:
        """No SMTP here: mails land in <root>/outbox (settings.py:165-170 had SMTP creds)."""
        d = os.path.join(settings.storage_root, "outbox")
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, f"{time.time():.6f}.eml"), "w", encoding="utf-8") as f:
            f.write(f"To: {to}\nSubject: {subject}\n\n{body}\n")

    html_auth.install(app, db, settings, outbox, validate_password, form, current_user)

    # ================================================================== /rest-auth/
    @app.post("/rest-auth/login/")
    async def login(request: Request):
        f, _, e = await form(request)
        if e:
            return e
        user = None
        if f.get("username"):
            user = db.find_user(username=f["username"])
        elif f.get("email"):
            user = db.find_user(email=f["email"])
        if not user or not check_password(str(f.get("password", "")), user["password"]):
            return J({"non_field_errors": ["Unable to log in with provided credentials."]}, 400)
        return J({"key": db.token_for(user["id"])})

    @app.post("/rest-auth/logout/")
    async def logout(request: Request):
        u = current_user(request)
        if u:
            db.delete_token(u["id"])
        return J({"detail": "Successfully logged out."})

    @app.post("/rest-auth/registration/")
    async def register(request: Request):
        f, _, e = await form(request)
        if e:
            return e
        username, email = str(f.get("username", "")).strip(), str(f.get("email", "")).strip()
        p1, p2 = str(f.get("password1", "")), str(f.get("password2", ""))
        errs: Dict[str, List[str]] = {}
        if not username:
            errs["username"] = ["This field is required."]
        elif db.find_user(username=username):
            errs["username"] = ["A user with that username already exists."]
        if email and db.find_user(email=email):
            errs["email"] = ["A user is already registered with this e-mail address."]
        if not p1:
            errs["password1"] = ["This field is required."]
        else:
            pe = validate_password(p1, username, email)
            if pe:
                errs["password1"] = pe
        if p1 != p2:
            errs["non_field_errors"] = ["The two password fields didn't match."]
        if errs:
            return J(errs, 400)
        uid = db.create_user(username, p1, email)
        if email:
            outbox(email, "Confirm your e-mail", f"key: {db.new_email_key(uid)}")
        return J({"key": db.token_for(uid)}, 201)

    @app.post("/rest-auth/registration/verify-email/")
    async def verify_email(request: Request):
        f, _, e = await form(request)
        if e:
            return e
        if db.verify_email_key(str(f.get("key", ""))) is None:
            return J({"detail": "Not found."}, 404)
        return J({"detail": "ok"})

    @app.post("/rest-auth/password/reset/")
    async def password_reset(request: Request):
        f, _, e = await form(request)
        if e:
            return e
        email = str(f.get("email", ""))
        if not email:
            return J({"email": ["This field is required."]}, 400)
        user = db.find_user(email=email)
        if user:
            tok = db.new_reset_token(user["id"])
            outbox(email, "Password reset", f"uid: {user['id']}\ntoken: {tok}")
        return J({"detail": "Password reset e-mail has been sent."})

    @app.post("/rest-auth/password/reset/confirm/")
    async def password_reset_confirm(request: Request):
        f, _, e = await form(request)
        if e:
            return e
        try:
            uid = int(f.get("uid", -1))
        except (TypeError, ValueError):
            uid = -1
        p1, p2 = str(f.get("new_password1", "")), str(f.get("new_password2", ""))
        user = db.get_user(uid)
        if not user or not db.use_reset_token(uid, str(f.get("token", ""))):
            return J({"token": ["Invalid value"]}, 400)
        if p1 != p2:
            return J({"new_password2": ["The two password fields didn't match."]}, 400)
        pe = validate_password(p1, user["username"], user["email"])
        if pe:
            return J({"new_password2": pe}, 400)
        db.set_password(uid, p1)
        return J({"detail": "Password has been reset with the new password."})

    @app.post("/rest-auth/password/change/")
    async def password_change(request: Request):
        u, e = need_user(request)
        if e:
            return e
        f, _, e = await form(request)
        if e:
            return e
        if "old_password" in f and not check_password(str(f["old_password"]), u["password"]):
            return J({"old_password": ["Invalid password"]}, 400)
        p1, p2 = str(f.get("new_password1", "")), str(f.get("new_password2", ""))
        if p1 != p2:
            return J({"new_password2": ["The two password fields didn't match."]}, 400)
        pe = validate_password(p1, u["username"], u["email"])
        if pe:
            return J({"new_password2": pe}, 400)
        db.set_password(u["id"], p1)        # revokes every session/token of the user ...
        # ... and this client gets a fresh one (Django's update_session_auth_hash)
        return J({"detail": "New password has been saved.", "key": db.token_for(u["id"])})

    @app.get("/rest-auth/user/")
    async def user_get(request: Request):
        u, e = need_user(request)
        return e or J(user_json(u))

    @app.api_route("/rest-auth/user/", methods=["PUT", "PATCH"])
    async def user_update(request: Request):
        u, e = need_user(request)
        if e:
            return e
        f, _, e = await form(request)
        if e:
            return e
        if request.method == "PUT" and not f.get("username"):
            return J({"username": ["This field is required."]}, 400)
        if "username" in f and f["username"] != u["username"] and db.find_user(username=f["username"]):
            return J({"username": ["A user with that username already exists."]}, 400)
        db.update_user(u["id"], **{k: str(v) for k, v in f.items() if k in ("username", "first_name", "last_name")})
        return J(user_json(db.get_user(u["id"])))

    # ================================================================== /data/
    @app.post("/data/create/")
    async def model_create(request: Request):
        u, e = need_user(request)
        if e:
            return e
        f, _, e = await form(request)
        if e:
            return e
        name = f.get("modelName")
        if not valid_name(name):
            return J({"message": "error"}, 500)
        d = settings.model_dir(u["id"], name)
        try:
            os.makedirs(os.path.dirname(d), exist_ok=True)
            os.mkdir(d)                                 # reference: error if it exists (os.mkdir)
        except OSError:
            return J({"message": "error"}, 500)
        return J({"message": "success"})

    @app.post("/data/tag/")
    async def tag_upload(request: Request):
        u, e = need_user(request)
        if e:
            return e
        f, files, e = await form(request)
        if e:
            return e
        name, up = f.get("modelName"), files.get("file")
        if not valid_name(name) or up is None:
            return J({"message": "error"}, 500)
        d = settings.model_dir(u["id"], name)
        if not os.path.isdir(d):
            return J({"message": "error"}, 500)
        try:
            tags = json.loads(up.data.decode("utf-8-sig"))
            if not isinstance(tags, dict):
                raise ValueError
        except (ValueError, UnicodeDecodeError):
            return J({"message": "error", "detail": "tag file must be a JSON object"}, 500)
        with open(os.path.join(d, "tag.json"), "wb") as out:
            out.write(up.data)
        return J({"message": "success"})

    def raw_json(r: Dict[str, Any]) -> Dict[str, Any]:
        return {"id": r["id"], "created_at": time.strftime("%Y-%m-%dT%H:%M:%S", time.localtime(r["created_at"])),
                "file_type": r["file_type"], "file_name": r["file_path"].rstrip("/").split("/")[-1],
                "owner": r["owner_id"]}

    @app.get("/data/list/")
    async def data_list(request: Request):
        u, e = need_user(request)
        return e or J([raw_json(r) for r in db.list_raw_data(u["id"])])

    @app.post("/data/list/")
    async def data_upload(request: Request):
        u, e = need_user(request)
        if e:
            return e
        f, files, e = await form(request)
        if e:
            return e
        ftype, fclass = f.get("file_type"), f.get("file_class", "picture")
        if ftype not in ("single", "zip", "url") or fclass not in FILE_TYPES:
            return J({"message": "error"}, 400)
        rel_dir = os.path.join("NJUCloud", str(u["id"]), "data", fclass)
        abs_dir = os.path.join(settings.storage_root, rel_dir)
        os.makedirs(abs_dir, exist_ok=True)
        try:
            if ftype in ("single", "zip"):
                up = files.get("file")
                if up is None:
                    return J({"message": "error"}, 400)
                base = os.path.basename(up.filename.replace("\\", "/")) or "upload"
                fname = timestamped_name(base)
                if ftype == "single":
                    with open(os.path.join(abs_dir, fname), "wb") as out:
                        out.write(up.data)
                    rel = os.path.join(rel_dir, fname)
                else:
                    stem = os.path.splitext(fname)[0]
                    dest = os.path.join(abs_dir, stem)
                    await run_in_threadpool(_extract_zip, up.data, dest)
                    rel = os.path.join(rel_dir, stem)
            else:
                if not settings.allow_url_fetch:
                    return J({"message": "error", "detail": "URL datasets are disabled"}, 400)
                urls = [x.strip() for x in str(f.get("url", "")).split(";") if x.strip()]
                if not urls:
                    return J({"message": "error"}, 400)
                try:
                    for url in urls:
                        net.check_url(url)       # http(s) only: refuse the whole request
                except net.FetchRefused as exc:
                    return J({"message": "error", "detail": str(exc)}, 400)
                stem = timestamped_name("url")
                dest = os.path.join(abs_dir, stem)
                os.makedirs(dest, exist_ok=True)
                errors = await run_in_threadpool(_fetch_urls, urls, dest, settings.url_allow_private,
                                                 max_bytes)
                if errors and len(errors) == len(urls):
                    shutil.rmtree(dest, ignore_errors=True)
                    return J({"message": "error", "detail": "; ".join(errors)}, 400)
                rel = os.path.join(rel_dir, stem)
        except (zipfile.BadZipFile, OSError, ValueError):
            return J({"message": "error"}, 500)
        return J({"data_id": db.add_raw_data(u["id"], rel, fclass)})

    def owned_raw(u, pk: int):
        r = db.get_raw_data(pk)
        if r is None:
            return None, J({"detail": "Not found."}, 404)
        if r["owner_id"] != u["id"]:
            return None, J({"detail": "You do not have permission to perform this action."}, 403)
        return r, None

    @app.get("/data/{pk}/")
    async def data_detail(pk: int, request: Request):
        u, e = need_user(request)
        if e:
            return e
        r, e = owned_raw(u, pk)
        if e:
            return e
        base = os.path.join(settings.storage_root, r["file_path"])
        rel = request.query_params.get("relative_path")
        path = safe_join(base, rel) if rel else base
        if path is None or not os.path.exists(path):
            return J({"detail": "Not found."}, 404)
        if path.endswith(".csv") and (rel is not None or r["file_type"] == "doc"):
            return Response(csv_to_json(path), media_type="application/json")
        if os.path.isfile(path):
            mt = mimetypes.guess_type(path)[0] or "application/octet-stream"
            with open(path, "rb") as fh:
                data = fh.read()
            return Response(data, media_type=mt, headers={
                "Content-Disposition": f"attachment; filename={os.path.basename(path)}"})
        return J(dir_tree(path))

    @app.delete("/data/{pk}/")
    async def data_delete(pk: int, request: Request):
        u, e = need_user(request)
        if e:
            return e
        r, e = owned_raw(u, pk)
        if e:
            return e
        db.delete_raw_data(pk)
        if request.query_params.get("purge") in ("1", "true"):
            p = os.path.join(settings.storage_root, r["file_path"])
            shutil.rmtree(p, ignore_errors=True) if os.path.isdir(p) else (os.path.exists(p) and os.remove(p))
        return J({"message": "success"})

    # ================================================================== /preprocess/
    @app.get("/preprocess/")
    async def preprocess_get(request: Request):
        return J({"message": "error"}, 501)

    @app.get("/preprocess/operations/list/")
    async def preprocess_ops(request: Request):
        return J([{"operationName": k, "op": v} for k, v in ops_ref.OP_MAP.items()])

    @app.post("/preprocess/")
    async def preprocess_post(request: Request):
        u, e = need_user(request)
        if e:
            return e
        f, _, e = await form(request)
        if e:
            return e
        try:
            data_id, model = int(f["dataId"]), f["modelName"]
            ops = f.get("operations") or []
            if isinstance(ops, str):
                ops = json.loads(ops)
        except (KeyError, TypeError, ValueError):
            return J({"message": "error"}, 500)
        if not valid_name(model):
            return J({"message": "error"}, 500)
        r, e = owned_raw(u, data_id)
        if e:
            return J({"message": "error"}, 500)
        mdir = settings.model_dir(u["id"], model)
        try:
            os.makedirs(mdir, exist_ok=True)
            await run_in_threadpool(pipeline.copy_dataset, os.path.join(settings.storage_root, r["file_path"]),
                                    os.path.join(mdir, "data"))
            tag = os.path.join(mdir, "tag.json")
            if ops:
                if not os.path.exists(tag):
                    return J({"message": "error", "detail": "upload tag.json first"}, 500)
                await run_in_threadpool(on_serve_device, pipeline.run, os.path.join(mdir, "data"), tag, ops,
                                        backend=settings.preprocess_backend)
        except Exception as exc:
            return J({"message": "error", "detail": str(exc)}, 500)
        return J({"message": "success"})

    # ================================================================== /construct/
    @app.post("/construct/options/")
    async def options(request: Request):
        f, _, e = await form(request)
        if e:
            return e
        try:
            return J(get_options(str(f.get("option"))))
        except KeyError:
            return J({"message": "error"}, 400)

    @app.get("/construct/config/")
    async def model_list(request: Request):
        u, e = need_user(request)
        if e:
            return e
        root = os.path.join(settings.user_root(u["id"]), "model")
        names = sorted(n for n in os.listdir(root) if os.path.isfile(os.path.join(root, n, RESULT))) \
            if os.path.isdir(root) else []
        return J(names)

    def read_model_json(uid: int, model: str):
        p = os.path.join(settings.model_dir(uid, model), "model.json")
        if not valid_name(model) or not os.path.exists(p):
            return None
        with open(p, encoding="utf-8") as fh:
            return json.load(fh)

    @app.get("/construct/detail/{model}/")
    async def model_detail(model: str, request: Request):
        u, e = need_user(request)
        if e:
            return e
        cfg = read_model_json(u["id"], model)
        return J(cfg) if cfg is not None else J({"detail": "Not found."}, 404)

    @app.post("/construct/construction/{model}/{datatype}/")
    async def construct(model: str, datatype: str, request: Request):
        u, e = need_user(request)
        if e:
            return e
        f, _, e = await form(request)
        if e:
            return e
        if not valid_name(model) or datatype not in ("url", "file"):
            return J({"message": "error", "detail": "bad model name or datatype"}, 400)
        try:
            cfg = parse_train_config(f)
        except ConfigError as exc:
            return J({"message": "error", "detail": str(exc)}, 400)
        ngpus = 1
        if isinstance(f.get("options"), dict):
            ngpus = int(f["options"].get("gpus", 1))
        try:
            jid = jobs.submit(u["id"], model, datatype, f, ngpus=ngpus)
        except JobConflict as exc:
            return J({"message": "error", "detail": str(exc)}, 409)
        except ValueError as exc:
            return J({"message": "error", "detail": str(exc)}, 400)
        return J({"message": "success", "job": jid, "params": cfg.plan().num_params()})

    @app.post("/construct/inference/{model}/")
    async def inference(model: str, request: Request):
        u, e = need_user(request)
        if e:
            return e
        f, files, e = await form(request)
        if e:
            return e
        up = files.get("file")
        if up is None or not valid_name(model):
            return J({"result": "fail", "message": "no file"}, 400)
        mdir = settings.model_dir(u["id"], model)
        if not os.path.isdir(mdir):
            return J(dict(FAIL_NO_MODEL))
        idir = os.path.join(mdir, "infer")

        def keep_upload():
            os.makedirs(idir, exist_ok=True)
            with open(os.path.join(idir, os.path.basename(up.filename) or "image"), "wb") as out:
                out.write(up.data)
        await run_in_threadpool(keep_upload)
        prep = str(request.query_params.get("prep", f.get("prep", "reference")))
        return J(await infer.predict_async(mdir, up.data, prep=prep))

    # ================================================================== /runtime/
    @app.get("/runtime/train/{model}/{iters}/")
    async def train_results(model: str, iters: int, request: Request):
        u, e = need_user(request)
        if e:
            return e
        if not valid_name(model):
            return J({"detail": "Not found."}, 404)
        return J(read_train_results(os.path.join(settings.model_dir(u["id"], model), RESULT), iters))

    @app.get("/runtime/kubernetes/")
    async def kubernetes(request: Request):
        u, e = need_user(request)
        if e:
            return e
        return J(node_status(db.active_jobs()))

    # ================================================================== /generation/ + /models/
    @app.get("/generation/options/list/")
    async def gen_options(request: Request):
        return J({k: dict(v) for k, v in CATALOG.items()})

    @app.get("/generation/options/next/")
    async def gen_next(request: Request):
        prev = request.query_params.get("layer", "")
        spatial = ["conv", "pool", "norm", "active", "connect"]
        flat = ["connect", "active"]
        return J({"options": flat if prev == "connect" else spatial})

    @app.post("/generation/generate/")
    async def gen_generate(request: Request):
        f, _, e = await form(request)
        if e:
            return e
        try:
            cfg = parse_train_config(f)
        except ConfigError as exc:
            return J({"message": "error", "detail": str(exc)}, 400)
        plan = cfg.plan()
        return J({"message": "success", "params": plan.num_params(), "flops_per_sample": plan.flops_per_sample(),
                  "layers": [{"index": lp.index, "spec": spec_to_dict(lp.spec),
                              "out": [lp.out_shape.c] + (list(lp.out_shape.hw) if lp.out_shape.hw else [])}
                             for lp in plan.layers]})

    def latest_job(uid: int, model: str):
        js = db.jobs_for(uid, model)
        return js[-1] if js else None

    async def model_arg(request: Request):
        f, _, e = await form(request)
        if e:
            return None, e
        m = f.get("modelName") or request.query_params.get("modelName")
        if not valid_name(m):
            return None, J({"message": "error", "detail": "modelName required"}, 400)
        return m, None

    @app.post("/generation/run/basic/")
    async def run_basic(request: Request):
        u, e = need_user(request)
        if e:
            return e
        m, e = await model_arg(request)
        if e:
            return e
        j = latest_job(u["id"], m)
        return J(jobs.status(j["id"]) if j else {"detail": "Not found."}, 200 if j else 404)

    @app.get("/generation/run/details/")
    async def run_details(request: Request):
        u, e = need_user(request)
        if e:
            return e
        m = request.query_params.get("modelName")
        if not valid_name(m):
            return J({"detail": "modelName required"}, 400)
        p = os.path.join(settings.model_dir(u["id"], m), METRICS)
        rows = []
        if os.path.exists(p):
            with open(p) as fh:
                rows = [json.loads(x) for x in fh if x.strip()]
        st = {}
        try:
            with open(os.path.join(settings.model_dir(u["id"], m), STATUS)) as fh:
                st = json.load(fh)
        except (OSError, json.JSONDecodeError):
            pass
        # the step program in use and, when it is not the HIP one, why (never silent)
        return J({"metrics": rows, "backend": st.get("backend"), "fallback_reason": st.get("fallback") or ""})

    @app.get("/generation/run/runtime/")
    async def run_runtime(request: Request):
        u, e = need_user(request)
        if e:
            return e
        m = request.query_params.get("modelName")
        if not valid_name(m):
            return J({"detail": "modelName required"}, 400)
        p = os.path.join(settings.model_dir(u["id"], m), STATUS)
        st = json.load(open(p)) if os.path.exists(p) else {}
        return J(st)

    async def control(request: Request, action: str):
        u, e = need_user(request)
        if e:
            return e
        m, e = await model_arg(request)
        if e:
            return e
        j = latest_job(u["id"], m)
        if j is None:
            return J({"detail": "Not found."}, 404)
        try:
            return J(jobs.control(j["id"], action))
        except ValueError as exc:
            return J({"message": "error", "detail": str(exc)}, 400)

    @app.post("/generation/run/stop/")
    async def run_stop(request: Request):
        return await control(request, "stop")

    @app.post("/generation/run/pause/")
    async def run_pause(request: Request):
        return await control(request, "pause")

    @app.get("/generation/restore/{jid}/")
    async def restore(jid: int, request: Request):
        u, e = need_user(request)
        if e:
            return e
        j = db.get_job(jid)
        if j is None or j["owner_id"] != u["id"]:
            return J({"detail": "Not found."}, 404)
        try:
            return J(jobs.control(jid, "resume"))
        except JobConflict as exc:
            return J({"message": "error", "detail": str(exc)}, 409)
        except ValueError as exc:
            return J({"message": "error", "detail": str(exc)}, 400)

    @app.get("/models/")
    async def models(request: Request):
        u, e = need_user(request)
        if e:
            return e
        root = os.path.join(settings.user_root(u["id"]), "model")
        out = []
        for n in sorted(os.listdir(root)) if os.path.isdir(root) else []:
            j = latest_job(u["id"], n)
            out.append({"name": n, "state": j["state"] if j else None, "job": j["id"] if j else None})
        return J(out)

    @app.get("/models/compare/")
    async def models_compare(request: Request):
        u, e = need_user(request)
        if e:
            return e
        names = [x for x in request.query_params.get("models", "").split(",") if valid_name(x)]
        out = {}
        for n in names:
            res = read_train_results(os.path.join(settings.model_dir(u["id"], n), RESULT), 0)
            out[n] = {"final_accuracy": res.get("final_accuracy"), "logged": len(res["every_result"])}
        return J(out)

    @app.get("/models/{model}/")
    async def model_get(model: str, request: Request):
        u, e = need_user(request)
        if e:
            return e
        cfg = read_model_json(u["id"], model)
        if cfg is None:
            return J({"detail": "Not found."}, 404)
        j = latest_job(u["id"], model)
        return J({"name": model, "config": cfg, "job": jobs.status(j["id"]) if j else None})

    @app.delete("/models/{model}/")
    async def model_delete(model: str, request: Request):
        u, e = need_user(request)
        if e:
            return e
        if not valid_name(model):
            return J({"detail": "Not found."}, 404)
        j = latest_job(u["id"], model)
        if j and j["state"] in ("queued", "running"):
            return J({"message": "error", "detail": "stop the job first"}, 409)
        shutil.rmtree(settings.model_dir(u["id"], model), ignore_errors=True)
        return J({"message": "success"})

    if settings.enable_demo:
        _install_demo(app, db, need_user, current_user, form)
    return app


def _install_metrics(app: FastAPI, db: Database) -> None:
    """Prometheus text exposition at /metrics: request counts/latency per route and the
    job table by state (the reference had print() only)."""
    try:
        import prometheus_client as prom
    except ImportError:       # pragma: no cover
        return
    reg = prom.CollectorRegistry()
    req = prom.Counter("csa_http_requests_total", "HTTP requests", ["method", "route", "status"], registry=reg)
    lat = prom.Histogram("csa_http_request_seconds", "HTTP request latency", ["route"], registry=reg)
    jobs_g = prom.Gauge("csa_jobs", "training jobs by state", ["state"], registry=reg)

    @app.middleware("http")
    async def _count(request: Request, call_next):
        t0 = time.perf_counter()
        resp = await call_next(request)
        route = request.scope.get("route")
        path = getattr(route, "path", "unmatched")
        req.labels(request.method, path, str(resp.status_code)).inc()
        lat.labels(path).observe(time.perf_counter() - t0)
        return resp

    @app.get("/metrics")
    async def metrics():
        counts: Dict[str, int] = {}
        for (st,) in db.conn().execute("SELECT state FROM jobs").fetchall():
            counts[st] = counts.get(st, 0) + 1
        for st in ("queued", "running", "paused", "stopped", "failed", "done"):
            jobs_g.labels(st).set(counts.get(st, 0))
        return Response(prom.generate_latest(reg), media_type=prom.CONTENT_TYPE_LATEST)


def _install_demo(app: FastAPI, db: Database, need_user, current_user, form) -> None:
    """The reference's scaffolding "Bills" app (demo/*.py; its routes are commented out
    in CloudServer/urls.py:25, so it is off unless CSA_ENABLE_DEMO=1).  Same paths:
    GET/POST /demo/, GET /demo/search/?name=, GET/PUT/DELETE /demo/<pk>/ with the
    owner-or-read-only rule of demo/permission.py:5-26."""

    def bill_json(b):
        return {k: b[k] for k in ("id", "goods", "price", "amount", "description", "owner")}

    def parse(f, partial=False):
        out = {}
        try:
            if "goods" in f or not partial:
                g = str(f.get("goods", "")).strip()
                if not g or len(g) > 100:
                    raise ValueError("goods")
                out["goods"] = g
            if "price" in f or not partial:
                out["price"] = float(f["price"])
            if "amount" in f:
                out["amount"] = int(f["amount"])
            if "description" in f:
                out["description"] = str(f["description"])[:100]
        except (KeyError, TypeError, ValueError) as exc:
            raise ValueError(str(exc))
        return out

    @app.get("/demo/")
    async def bills_list(request: Request):
        return J([bill_json(b) for b in db.list_bills()])

    @app.post("/demo/")
    async def bills_create(request: Request):
        u, e = need_user(request)
        if e:
            return e
        f, _, e = await form(request)
        if e:
            return e
        try:
            fields = parse(f)
        except ValueError as exc:
            return J({"detail": f"invalid field {exc}"}, 400)
        return J(bill_json(db.get_bill(db.add_bill(u["id"], **fields))), 201)

    @app.get("/demo/search/")
    async def bills_search(request: Request):
        return J([bill_json(b) for b in db.list_bills(request.query_params.get("name", ""))])

    @app.api_route("/demo/{pk}/", methods=["GET", "PUT", "DELETE"])
    async def bill_detail(pk: int, request: Request):
        b = db.get_bill(pk)
        if b is None:
            return J({"detail": "Not found."}, 404)
        if request.method == "GET":
            return J(bill_json(b))
        u, e = need_user(request)
        if e:
            return e
        if u["id"] != b["owner_id"]:
            return J({"detail": "You do not have permission to perform this action."}, 403)
        if request.method == "DELETE":
            db.delete_bill(pk)
            return Response(status_code=204)
        f, _, e = await form(request)
        if e:
            return e
        try:
            db.update_bill(pk, **parse(f))
        except ValueError as exc:
            return J({"detail": f"invalid field {exc}"}, 400)
        return J(bill_json(db.get_bill(pk)))


def _fetch_urls(urls: List[str], dest: str, allow_private: bool, max_bytes: int) -> List[str]:
    """Sequential downloads (apps/data/views.py:193-208), each through the SSRF guard;
    a failing URL is reported and the others continue (the reference logged and went on)."""
    errors = []
    for url in urls:
        name = os.path.basename(url.split("?", 1)[0].rstrip("/")) or "download"
        if not valid_name(name):
            name = "download"
        try:
            net.fetch(url, os.path.join(dest, name), allow_private=allow_private, max_bytes=max_bytes)
        except (net.FetchRefused, OSError, ValueError) as exc:
            errors.append(f"{url}: {exc}")
    return errors


def _extract_zip(data: bytes, dest: str) -> None:
    """Extract with the reference's cp437 -> utf8 name fix (views.py:150-162), refusing
    members that would land outside ``dest`` (zip-slip)."""
    os.makedirs(dest, exist_ok=True)
    with zipfile.ZipFile(io.BytesIO(data)) as z:
        for info in z.infolist():
            name = info.filename
            if not (info.flag_bits & 0x800):
                try:
                    name = name.encode("cp437").decode("utf-8")
                except (UnicodeEncodeError, UnicodeDecodeError):
                    pass
            target = safe_join(dest, name)
            if target is None:
                continue
            if name.endswith("/"):
                os.makedirs(target, exist_ok=True)
                continue
            os.makedirs(os.path.dirname(target), exist_ok=True)
            with z.open(info) as src, open(target, "wb") as out:
                shutil.copyfileobj(src, out)


def main() -> None:   # pragma: no cover - CLI
    import argparse
    import uvicorn
    ap = argparse.ArgumentParser(prog="cloud_server_amd.api.app")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8000)
    a = ap.parse_args()
    uvicorn.run(create_app(), host=a.host, port=a.port)


if __name__ == "__main__":   # pragma: no cover
    main()

"""End-to-end REST API tests (CPU): the user flow of SURVEY.md §3.1 through FastAPI's
TestClient — register/login, upload a zip of digit PNGs + tag.json, preprocess, build a
model from the DSL, train it (inline executor), poll results, list/detail models, infer.

Reference parity: apps/*/views.py behaviour and API.md payloads; data is synthetic
(reference test-data images are PNGs loaded with PIL, not pickles)."""
import base64
import io
import json
import os
import zipfile

import numpy as np
import pytest
from fastapi.testclient import TestClient
from PIL import Image

from cloud_server_amd.api.app import create_app, validate_password
from cloud_server_amd.api.forms import encode_multipart, parse_multipart
from cloud_server_amd.config import Settings
from cloud_server_amd.data.datasets import synthetic_mnist

PW = "Str0ng-pass-42"


def _png(arr):
    b = io.BytesIO()
    Image.fromarray(arr.astype(np.uint8)).save(b, format="PNG")
    return b.getvalue()


@pytest.fixture()
def client(tmp_path):
    s = Settings(storage_root=str(tmp_path / "store"), db_path=str(tmp_path / "db.sqlite3"),
                 executor="inline", train_backend="torch", allow_url_fetch=True)
    app = create_app(s, executor="inline", ngpu=0, inference_device="cpu")
    with TestClient(app) as c:
        c.settings = s
        yield c


def _auth(c, name="alice"):
    r = c.post("/rest-auth/registration/", json={"username": name, "email": f"{name}@x.org",
                                                   "password1": PW, "password2": PW})
    assert r.status_code == 201, r.text
    r = c.post("/rest-auth/login/", json={"username": name, "password": PW})
    assert r.status_code == 200
    return {"Authorization": "Token " + r.json()["key"]}


def _mp(c, url, fields, files, headers):
    body, ct = encode_multipart(fields, files)
    return c.post(url, content=body, headers={**headers, "Content-Type": ct})


def _digit_zip(n=60):
    ds = synthetic_mnist(n, seed=3)
    zb = io.BytesIO()
    tags = {}
    with zipfile.ZipFile(zb, "w") as z:
        for i in range(n):
            name = f"img_{i:03d}.png"
            z.writestr(f"digits/{name}", _png(ds.images[i].reshape(28, 28)))
            tags[f"digits/{name}"] = int(ds.labels[i])
    return zb.getvalue(), tags, ds


def test_password_validators():
    assert validate_password("short")
    assert validate_password("12345678901")
    assert validate_password("password")
    assert validate_password("alice-the-great", "alice")
    assert not validate_password(PW, "bob", "bob@x.org")


def test_multipart_roundtrip():
    body, ct = encode_multipart({"a": "1", "b": "héllo"}, {"file": ("x.bin", b"\x00\r\n--x\xff", "application/x")})
    f, files = parse_multipart(body, ct)
    assert f == {"a": "1", "b": "héllo"}
    assert files["file"].data == b"\x00\r\n--x\xff" and files["file"].filename == "x.bin"


def test_auth_flow(client):
    h = _auth(client)
    r = client.get("/rest-auth/user/", headers=h)
    assert r.status_code == 200 and r.json()["username"] == "alice"
    assert client.get("/rest-auth/user/").status_code == 401
    basic = {"Authorization": "Basic " + base64.b64encode(f"alice:{PW}".encode()).decode()}
    assert client.get("/rest-auth/user/", headers=basic).status_code == 200
    r = client.patch("/rest-auth/user/", json={"first_name": "Al"}, headers=h)
    assert r.json()["first_name"] == "Al"
    # duplicate / weak registration
    r = client.post("/rest-auth/registration/", json={"username": "alice", "password1": "x", "password2": "y"})
    assert r.status_code == 400 and "username" in r.json()
    # bad login
    assert client.post("/rest-auth/login/", json={"username": "alice", "password": "nope"}).status_code == 400
    # password change
    new = "An0ther-pass-77"
    r = client.post("/rest-auth/password/change/", json={"old_password": PW, "new_password1": new,
                                                         "new_password2": new}, headers=h)
    assert r.status_code == 200
    assert client.post("/rest-auth/login/", json={"username": "alice", "password": new}).status_code == 200
    # reset via outbox mail
    assert client.post("/rest-auth/password/reset/", json={"email": "alice@x.org"}).status_code == 200
    box = os.path.join(client.settings.storage_root, "outbox")
    mail = [open(os.path.join(box, f)).read() for f in sorted(os.listdir(box)) if "reset" in open(os.path.join(box, f)).read()][-1]
    uid = mail.split("uid: ")[1].split()[0]
    tok = mail.split("token: ")[1].split()[0]
    third = "Thr33-pass-xyz"
    r = client.post("/rest-auth/password/reset/confirm/", json={"uid": uid, "token": tok,
                                                                "new_password1": third, "new_password2": third})
    assert r.status_code == 200, r.text
    # token is single-use
    r = client.post("/rest-auth/password/reset/confirm/", json={"uid": uid, "token": tok,
                                                                "new_password1": third, "new_password2": third})
    assert r.status_code == 400
    # logout invalidates the token
    h2 = {"Authorization": "Token " + client.post("/rest-auth/login/", json={"username": "alice", "password": third}).json()["key"]}
    assert client.post("/rest-auth/logout/", headers=h2).status_code == 200
    assert client.get("/rest-auth/user/", headers=h2).status_code == 401


def test_data_upload_detail_delete(client):
    h = _auth(client)
    hb = _auth(client, "bob")
    # single csv doc
    r = _mp(client, "/data/list/", {"file_type": "single", "file_class": "doc"},
            {"file": ("t.csv", b"a,b\n1,2\n3,4\n", "text/csv")}, h)
    assert r.status_code == 200, r.text
    pk = r.json()["data_id"]
    r = client.get(f"/data/{pk}/", headers=h)
    assert r.json() == [{"a": "1", "b": "2"}, {"a": "3", "b": "4"}]
    lst = client.get("/data/list/", headers=h).json()
    assert len(lst) == 1 and lst[0]["file_type"] == "doc" and lst[0]["file_name"].startswith("t_") and lst[0]["file_name"].endswith(".csv")
    # zip picture: tree listing + relative file download
    zb, tags, _ = _digit_zip(4)
    r = _mp(client, "/data/list/", {"file_type": "zip", "file_class": "picture"},
            {"file": ("digits.zip", zb, "application/zip")}, h)
    zpk = r.json()["data_id"]
    tree = client.get(f"/data/{zpk}/", headers=h).json()
    assert "digits" in json.dumps(tree)
    r = client.get(f"/data/{zpk}/", params={"relative_path": "digits/img_000.png"}, headers=h)
    assert r.status_code == 200 and r.content[:4] == b"\x89PNG"
    # path escape refused
    r = client.get(f"/data/{zpk}/", params={"relative_path": "../../../../db.sqlite3"}, headers=h)
    assert r.status_code == 404
    # other users cannot read or delete
    assert client.get(f"/data/{pk}/", headers=hb).status_code == 403
    assert client.delete(f"/data/{pk}/", headers=hb).status_code == 403
    assert client.delete(f"/data/{pk}/", headers=h).status_code == 200
    assert client.get(f"/data/{pk}/", headers=h).status_code == 404
    assert client.get("/data/list/").status_code == 401


def test_zip_slip_refused(client):
    h = _auth(client)
    zb = io.BytesIO()
    with zipfile.ZipFile(zb, "w") as z:
        z.writestr("../../evil.txt", b"x")
        z.writestr("ok.txt", b"y")
    r = _mp(client, "/data/list/", {"file_type": "zip", "file_class": "doc"},
            {"file": ("e.zip", zb.getvalue(), "application/zip")}, h)
    assert r.status_code == 200
    assert not os.path.exists(os.path.join(client.settings.storage_root, "NJUCloud", "1", "evil.txt"))


def test_options_and_generate(client):
    r = client.post("/construct/options/", json={"option": "optimizer"})
    assert r.status_code == 200 and r.json()["tokens"]["Adam Optimizer"] == "AdamOptimizer"
    assert client.post("/construct/options/", json={"option": "nope"}).status_code == 400
    r = client.post("/generation/generate/", json={"iter": 5, "learning_rate": 0.1, "ratio": 0.8,
                                                   "net_config": {"middle_layer": [{"layer": "connect", "hidden": 32}]}})
    assert r.status_code == 200, r.text
    assert r.json()["params"] == 784 * 32 + 32 + 32 * 10 + 10
    assert client.get("/preprocess/").status_code == 501
    assert len(client.get("/preprocess/operations/list/").json()) == 14


def test_full_user_flow(client):
    h = _auth(client)
    zb, tags, ds = _digit_zip(60)
    assert client.post("/data/create/", json={"modelName": "m1"}, headers=h).json() == {"message": "success"}
    assert client.post("/data/create/", json={"modelName": "m1"}, headers=h).status_code == 500
    assert client.post("/data/create/", json={"modelName": "../x"}, headers=h).status_code == 500
    r = _mp(client, "/data/tag/", {"modelName": "m1"}, {"file": ("tag.json", json.dumps(tags).encode(), "application/json")}, h)
    assert r.json() == {"message": "success"}
    pk = _mp(client, "/data/list/", {"file_type": "zip", "file_class": "picture"},
             {"file": ("d.zip", zb, "application/zip")}, h).json()["data_id"]
    ops = [{"operationName": "左右翻转", "overlap": True},
           {"operationName": "对比度亮度调整", "value1": 1.2, "value2": 5, "overlap": "true"}]
    r = client.post("/preprocess/", json={"dataId": pk, "modelName": "m1", "operations": ops}, headers=h)
    assert r.json() == {"message": "success"}, r.text
    mdir = client.settings.model_dir(1, "m1")
    newtags = json.load(open(os.path.join(mdir, "tag.json")))
    assert len(newtags) == 60 * 3    # originals + one copy per op (batch mode)
    cfg = {"iter": 40, "learning_rate": 0.05, "ratio": 0.8, "loss_name": "entropy",
           "optimizer_name": "AdamOptimizer", "net_type": "CNN",
           "options": {"log_every": 10, "ckpt_every": 20, "batch_size": 16},
           "net_config": {"middle_layer": [{"layer": "conv", "filter": [3, 3, 4]},
                                           {"layer": "active", "active_func": "relu"},
                                           {"layer": "pool"},
                                           {"layer": "connect", "hidden": 16}], "output_layer": {}}}
    r = client.post("/construct/construction/m1/file/", json=cfg, headers=h)
    assert r.status_code == 200, r.text
    jid = r.json()["job"]
    assert client.app.state.jobs.wait(jid, 300) == "done"
    res = client.get("/runtime/train/m1/40/", headers=h).json()
    assert len(res["every_result"]) == 5 and 0.0 <= float(res["final_accuracy"]) <= 1.0   # 0..40
    assert client.get("/construct/config/", headers=h).json() == ["m1"]
    assert client.get("/construct/detail/m1/", headers=h).json()["iter"] == 40
    assert client.get("/construct/detail/zz/", headers=h).status_code == 404
    models = client.get("/models/", headers=h).json()
    assert models[0]["name"] == "m1" and models[0]["state"] == "done"
    assert client.get("/models/m1/", headers=h).json()["job"]["state"] == "done"
    assert "m1" in client.get("/models/compare/", params={"models": "m1"}, headers=h).json()
    det = client.get("/generation/run/details/", params={"modelName": "m1"}, headers=h).json()
    assert len(det["metrics"]) >= 4
    assert det["backend"] == "torch" and det["fallback_reason"] == ""      # (CPU: the eager program)
    assert client.get("/generation/run/runtime/", params={"modelName": "m1"}, headers=h).json()["state"] == "done"
    img = _png(ds.images[0].reshape(28, 28))
    r = _mp(client, "/construct/inference/m1/", {}, {"file": ("q.png", img, "image/png")}, h)
    out = r.json()
    assert out["result"] == "success" and out["message"] in list("0123456789")
    r = _mp(client, "/construct/inference/none/", {}, {"file": ("q.png", img, "image/png")}, h)
    assert r.json()["result"] == "fail"
    node = client.get("/runtime/kubernetes/", headers=h).json()
    assert {"Conditions", "Capacity", "Allocatable", "System Info", "Non-terminated Pods"} <= set(node)
    assert client.delete("/models/m1/", headers=h).json() == {"message": "success"}
    assert client.get("/models/", headers=h).json() == []


def test_construct_rejects_bad_config(client):
    h = _auth(client)
    r = client.post("/construct/construction/m2/file/", json={"iter": 5, "net_config": {"middle_layer": [{"layer": "conv"}]}}, headers=h)
    assert r.status_code == 400
    r = client.post("/construct/construction/m2/ftp/", json={"iter": 5, "net_config": {"middle_layer": []}}, headers=h)
    assert r.status_code == 400


def test_metrics_cors_and_demo(tmp_path):
    s = Settings(storage_root=str(tmp_path / "store"), db_path=str(tmp_path / "db.sqlite3"),
                 executor="inline", train_backend="torch", cors_origins=["http://ui.example"], enable_demo=True)
    with TestClient(create_app(s, executor="inline", ngpu=0, inference_device="cpu")) as c:
        h = _auth(c)
        hb = _auth(c, "bob")
        r = c.options("/data/list/", headers={"Origin": "http://ui.example", "Access-Control-Request-Method": "POST",
                                              "Access-Control-Request-Headers": "authorization"})
        assert r.headers.get("access-control-allow-origin") == "http://ui.example"
        m = c.get("/metrics").text
        assert "csa_http_requests_total" in m and 'csa_jobs{state="running"}' in m
        # demo bills: list/create/search/detail with owner-or-read-only
        assert c.post("/demo/", json={"goods": "apple", "price": 2.5}).status_code == 401
        b = c.post("/demo/", json={"goods": "apple", "price": 2.5, "amount": 3}, headers=h).json()
        assert b["owner"] == "alice" and b["amount"] == 3
        c.post("/demo/", json={"goods": "pear", "price": 1}, headers=hb)
        assert [x["goods"] for x in c.get("/demo/").json()] == ["apple", "pear"]
        assert [x["goods"] for x in c.get("/demo/search/", params={"name": "pp"}).json()] == ["apple"]
        assert c.get(f"/demo/{b['id']}/").json()["price"] == 2.5
        assert c.put(f"/demo/{b['id']}/", json={"goods": "apple", "price": 3}, headers=hb).status_code == 403
        assert c.put(f"/demo/{b['id']}/", json={"goods": "apple", "price": 3}, headers=h).json()["price"] == 3
        assert c.delete(f"/demo/{b['id']}/", headers=h).status_code == 204
        assert c.get(f"/demo/{b['id']}/").status_code == 404


class _FixtureServer:
    """Serves a directory over http on 127.0.0.1 (URL datasets need http(s))."""

    def __init__(self, root):
        import functools
        import http.server
        import threading
        h = functools.partial(http.server.SimpleHTTPRequestHandler, directory=str(root))
        h.log_message = lambda *a, **k: None
        self.httpd = http.server.ThreadingHTTPServer(("127.0.0.1", 0), h)
        self.port = self.httpd.server_address[1]
        self.t = threading.Thread(target=self.httpd.serve_forever, daemon=True)
        self.t.start()

    def close(self):
        self.httpd.shutdown()
        self.httpd.server_close()


def test_url_dataset_and_url_training(client, tmp_path):
    """datatype=url: ';'-separated URLs downloaded into the dataset (a local http server
    here — no network; private destinations are opted in for the test), then the
    MNIST-idx training variant (construct_distribute_url.py)."""
    from cloud_server_amd.data.datasets import write_idx
    src = tmp_path / "mnist"
    src.mkdir()
    tr, te = synthetic_mnist(300, seed=5), synthetic_mnist(100, seed=6)
    import gzip
    for stem, arr in [("train-images-idx3-ubyte", tr.images.reshape(-1, 28, 28)),
                      ("train-labels-idx1-ubyte", tr.labels.astype(np.uint8)),
                      ("t10k-images-idx3-ubyte", te.images.reshape(-1, 28, 28)),
                      ("t10k-labels-idx1-ubyte", te.labels.astype(np.uint8))]:
        write_idx(str(src / stem), arr)
        with open(src / stem, "rb") as f, gzip.open(str(src / (stem + ".gz")), "wb") as g:
            g.write(f.read())
        os.remove(src / stem)
    srv = _FixtureServer(src)
    try:
        urls = ";".join(f"http://127.0.0.1:{srv.port}/{n}" for n in sorted(os.listdir(src)))
        h = _auth(client)
        client.settings.url_allow_private = True
        pk = _mp(client, "/data/list/", {"file_type": "url", "file_class": "picture", "url": urls}, {}, h).json()["data_id"]
    finally:
        srv.close()
    tree = json.dumps(client.get(f"/data/{pk}/", headers=h).json())
    assert "t10k-images-idx3-ubyte.gz" in tree
    client.post("/data/create/", json={"modelName": "mu"}, headers=h)
    assert client.post("/preprocess/", json={"dataId": pk, "modelName": "mu", "operations": []},
                       headers=h).json() == {"message": "success"}
    cfg = {"iter": 20, "learning_rate": 0.01, "optimizer_name": "AdamOptimizer", "options": {"log_every": 10},
           "net_config": {"middle_layer": [{"layer": "connect", "hidden": 32}]}}
    jid = client.post("/construct/construction/mu/url/", json=cfg, headers=h).json()["job"]
    assert client.app.state.jobs.wait(jid, 300) == "done"
    res = client.get("/runtime/train/mu/20/", headers=h).json()
    assert len(res["every_result"]) == 3 and "final_accuracy" in res      # 0, 10, 20


def test_url_fetch_refuses_file_and_private(client, tmp_path):
    """file:// (server files: the DB, the outbox) and loopback/private
    destinations are refused; only http(s) to public addresses is fetched."""
    from cloud_server_amd.utils import net
    secret = tmp_path / "secret.txt"
    secret.write_text("token")
    h = _auth(client)
    for url in (f"file://{secret}", "ftp://example.org/x", "gopher://x/"):
        r = _mp(client, "/data/list/", {"file_type": "url", "file_class": "doc", "url": url}, {}, h)
        assert r.status_code == 400, url
    srv = _FixtureServer(tmp_path)
    try:
        client.settings.url_allow_private = False
        r = _mp(client, "/data/list/", {"file_type": "url", "file_class": "doc",
                                        "url": f"http://127.0.0.1:{srv.port}/secret.txt"}, {}, h)
        assert r.status_code == 400 and "not allowed" in r.json()["detail"]
    finally:
        srv.close()
    assert client.get("/data/list/", headers=h).json() == []
    for a in ("127.0.0.1", "10.1.2.3", "192.168.0.1", "169.254.169.254", "::1", "::ffff:127.0.0.1", "0.0.0.0"):
        assert not net.address_allowed(a, False), a
    assert net.address_allowed("8.8.8.8", False)


def test_password_change_revokes_tokens(client):
    """a password change/reset revokes existing tokens and reset links."""
    h = _auth(client)
    db = client.app.state.db
    tok_old = db.new_reset_token(1)
    new = "An0ther-pass-77"
    r = client.post("/rest-auth/password/change/", json={"old_password": PW, "new_password1": new,
                                                         "new_password2": new}, headers=h)
    assert r.status_code == 200 and r.json()["key"]
    assert client.get("/rest-auth/user/", headers=h).status_code == 401          # old token revoked
    h2 = {"Authorization": "Token " + r.json()["key"]}
    assert client.get("/rest-auth/user/", headers=h2).status_code == 200
    assert not db.use_reset_token(1, tok_old)                                     # old reset link revoked


def _csrf(c, path):
    import re
    html = c.get(path).text
    return re.search(r"name='csrfmiddlewaretoken' value='([0-9a-f]+)'", html).group(1)


def test_browser_auth_pages_and_admin(client):
    """django.contrib.auth.urls + admin analogues: form login sets a session cookie that
    the JSON API accepts; password change / reset by form; /admin/ is staff-only; every
    form POST and every cookie-authenticated unsafe API call needs the CSRF token."""
    db = client.app.state.db
    uid = db.create_user("webu", PW, "webu@x.org")
    db.create_user("boss", PW, "boss@x.org", is_staff=True)
    assert "<form" in client.get("/login/").text
    tok = _csrf(client, "/login/")
    # login CSRF: a form post without the token is refused
    r = client.post("/login/", data={"username": "webu", "password": PW}, follow_redirects=False)
    assert r.status_code == 403
    r = client.post("/login/", data={"username": "webu", "password": "nope", "csrfmiddlewaretoken": tok},
                    follow_redirects=False)
    assert r.status_code == 200 and "correct username" in r.text
    r = client.post("/login/?next=//evil.example/", data={"username": "webu", "password": PW,
                                                         "csrfmiddlewaretoken": tok}, follow_redirects=False)
    assert r.status_code == 302 and r.headers["location"] == "/" and "sessionid" in r.cookies
    assert client.get("/rest-auth/user/").json()["username"] == "webu"     # session auth on the API
    # cookie-authenticated unsafe API call: needs X-CSRFToken == csrftoken cookie
    assert client.patch("/rest-auth/user/", json={"first_name": "W"}).status_code == 401
    ctok = client.cookies.get("csrftoken")
    r = client.patch("/rest-auth/user/", json={"first_name": "W"}, headers={"X-CSRFToken": ctok})
    assert r.status_code == 200 and r.json()["first_name"] == "W"
    assert client.get("/admin/", follow_redirects=False).status_code == 302  # not staff
    new = PW + "-2"
    tok = _csrf(client, "/password_change/")
    r = client.post("/password_change/", data={"old_password": PW, "new_password1": new,
                                               "new_password2": new, "csrfmiddlewaretoken": tok},
                    follow_redirects=False)
    assert r.status_code == 302 and r.headers["location"] == "/password_change/done/"
    assert client.get("/rest-auth/user/").json()["username"] == "webu"     # re-issued session
    # GET /logout/ only shows the confirmation form; the POST logs out
    assert "<form" in client.get("/logout/").text
    assert client.get("/rest-auth/user/").status_code == 200
    tok = _csrf(client, "/logout/")
    assert "Logged out" in client.post("/logout/", data={"csrfmiddlewaretoken": tok}).text
    client.cookies.clear()
    assert client.get("/rest-auth/user/").status_code == 401
    assert client.get("/password_change/", follow_redirects=False).status_code == 302
    # reset by e-mail link
    tok = _csrf(client, "/password_reset/")
    r = client.post("/password_reset/", data={"email": "webu@x.org", "csrfmiddlewaretoken": tok},
                    follow_redirects=False)
    assert r.headers["location"] == "/password_reset/done/"
    box = os.path.join(client.settings.storage_root, "outbox")
    mail = open(os.path.join(box, sorted(os.listdir(box))[-1])).read()
    link = [w for w in mail.split() if w.startswith("/reset/")][0]
    newer = PW + "-3"
    tok = _csrf(client, link)
    r = client.post(link, data={"new_password1": newer, "new_password2": newer, "csrfmiddlewaretoken": tok},
                    follow_redirects=False)
    assert r.status_code == 302 and r.headers["location"] == "/reset/done/"
    r = client.post(link, data={"new_password1": newer, "new_password2": newer, "csrfmiddlewaretoken": tok})
    assert r.status_code == 400  # one-shot
    assert client.post("/rest-auth/login/", data={"username": "webu", "password": newer}).status_code == 200
    # staff admin index
    tok = _csrf(client, "/login/")
    client.post("/login/", data={"username": "boss", "password": PW, "csrfmiddlewaretoken": tok})
    r = client.get("/admin/")
    assert r.status_code == 200 and "Site administration" in r.text and "users" in r.text
    assert uid


def test_event_loop_free_during_slow_preprocess(client, monkeypatch):
    """A slow /preprocess/ (dataset copy + pipeline run in the threadpool) does not stall
    other requests: GET /data/list/ answers in < 100 ms while it runs."""
    import asyncio
    import time
    import httpx
    from cloud_server_amd.preprocess import pipeline
    h = _auth(client)
    zb, tags, _ = _digit_zip(8)
    r = _mp(client, "/data/list/", {"file_type": "zip", "file_class": "picture"},
            {"file": ("d.zip", zb, "application/zip")}, h)
    pk = r.json()["data_id"]
    real = pipeline.copy_dataset

    def slow_copy(src, dst):
        time.sleep(1.5)
        return real(src, dst)
    monkeypatch.setattr(pipeline, "copy_dataset", slow_copy)

    async def go():
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=client.app), base_url="http://t") as ac:
            body, ct = encode_multipart({"dataId": str(pk), "modelName": "m"}, {})
            slow = asyncio.create_task(ac.post("/preprocess/", content=body, headers={**h, "Content-Type": ct}))
            await asyncio.sleep(0.2)             # the copy is now sleeping in a worker thread
            t0 = time.perf_counter()
            lst = await ac.get("/data/list/", headers=h)
            dt = time.perf_counter() - t0
            done_early = slow.done()
            res = await slow
            return lst, dt, done_early, res
    lst, dt, done_early, res = asyncio.run(go())
    assert lst.status_code == 200 and len(lst.json()) == 1
    assert not done_early and res.json()["message"] == "success", res.text
    assert dt < 0.1, dt


def test_construct_twice_is_409_and_result_stays_clean(tmp_path):
    """One job per (user, model): a second construct while the first is running gets 409
    (reference: the second launch pkill'ed the first, apps/construction/views.py:128-129)."""
    s = Settings(storage_root=str(tmp_path / "store"), db_path=str(tmp_path / "db.sqlite3"),
                 executor="thread", train_backend="torch")
    with TestClient(create_app(s, executor="thread", ngpu=0, inference_device="cpu")) as c:
        h = _auth(c)
        zb, tags, _ = _digit_zip(40)
        assert c.post("/data/create/", json={"modelName": "m"}, headers=h).json() == {"message": "success"}
        _mp(c, "/data/tag/", {"modelName": "m"}, {"file": ("tag.json", json.dumps(tags).encode(), "application/json")}, h)
        pk = _mp(c, "/data/list/", {"file_type": "zip", "file_class": "picture"},
                 {"file": ("d.zip", zb, "application/zip")}, h).json()["data_id"]
        assert c.post("/preprocess/", json={"dataId": pk, "modelName": "m", "operations": []}, headers=h).status_code == 200
        cfg = {"iter": 200, "learning_rate": 0.05, "ratio": 0.8, "optimizer_name": "AdamOptimizer",
               "options": {"log_every": 50, "ckpt_every": 0, "batch_size": 8},
               "net_config": {"middle_layer": [{"layer": "connect", "hidden": 16}]}}
        r1 = c.post("/construct/construction/m/file/", json=cfg, headers=h)
        r2 = c.post("/construct/construction/m/file/", json=cfg, headers=h)
        assert r1.status_code == 200 and r2.status_code == 409, (r1.text, r2.text)
        assert c.app.state.jobs.wait(r1.json()["job"], 300) == "done"
        res = c.get("/runtime/train/m/200/", headers=h).json()
        assert [r["step"] for r in res["every_result"]] == ["0", "50", "100", "150", "200"]
        assert "final_accuracy" in res
        assert len(c.app.state.db.jobs_for(1, "m")) == 1

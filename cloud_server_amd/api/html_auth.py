"""Browser (HTML form) auth pages and the admin index — the routes the reference gets
from ``django.contrib.auth.urls`` and ``admin.site.urls`` (CloudServer/urls.py:23,27;
SURVEY.md §2.7 rows `/login/ …` and `/admin/`).

* ``/login/`` ``/logout/`` — form login; the session cookie ``sessionid`` carries an API
  token, so a logged-in browser can also call the JSON API (``current_user`` accepts it,
  with Django's CSRF rule for unsafe methods: ``X-CSRFToken`` must match the
  ``csrftoken`` cookie).  Every form carries a ``csrfmiddlewaretoken`` field checked
  against that cookie (login CSRF included); ``/logout/`` only acts on a POST;
* ``/password_change/`` (+ ``done/``) — needs the session;
* ``/password_reset/`` (+ ``done/``), ``/reset/<uid>/<token>/`` (+ ``/reset/done/``) —
  the e-mail lands in ``<storage>/outbox`` (no SMTP here);
* ``/admin/`` — staff-only index; the reference registers no models (apps/*/admin.py are
  empty), so it lists the platform's tables read-only with row counts.

Pages are plain server-rendered HTML with every user value escaped.
"""
from __future__ import annotations

import hmac
import html
import secrets
from typing import Any, Callable, Dict, List, Optional

from fastapi import FastAPI, Request
from fastapi.responses import HTMLResponse, RedirectResponse

COOKIE = "sessionid"
CSRF_COOKIE = "csrftoken"
SESSION_AGE_S = 14 * 86400          # Django's SESSION_COOKIE_AGE


def _page(title: str, body: str, status: int = 200) -> HTMLResponse:
    return HTMLResponse(f"<!doctype html><html><head><meta charset='utf-8'><title>{html.escape(title)}"
                        f"</title></head><body><h1>{html.escape(title)}</h1>{body}</body></html>", status)


def csrf_token(request: Request) -> str:
    """The request's CSRF cookie value, or a fresh one (set by ``_with_csrf``)."""
    tok = request.cookies.get(CSRF_COOKIE, "")
    return tok if len(tok) >= 32 else secrets.token_hex(16)


def _with_csrf(resp, request: Request, tok: str):
    if request.cookies.get(CSRF_COOKIE) != tok:
        resp.set_cookie(CSRF_COOKIE, tok, samesite="lax", max_age=365 * 86400)
    return resp


def csrf_ok(request: Request, fields: Dict[str, Any]) -> bool:
    cookie = request.cookies.get(CSRF_COOKIE, "")
    sent = str(fields.get("csrfmiddlewaretoken", "") or request.headers.get("x-csrftoken", ""))
    return bool(cookie) and hmac.compare_digest(cookie, sent)


def _form(action: str, fields: List[tuple], submit: str, errors: Optional[List[str]] = None,
          csrf: str = "") -> str:
    err = "".join(f"<p class='error'>{html.escape(e)}</p>" for e in (errors or []))
    rows = "".join(f"<p><label>{html.escape(label)} <input type='{typ}' name='{name}'></label></p>"
                   for name, label, typ in fields)
    hidden = f"<input type='hidden' name='csrfmiddlewaretoken' value='{html.escape(csrf)}'>"
    return (f"{err}<form method='post' action='{html.escape(action)}'>{hidden}{rows}"
            f"<button>{html.escape(submit)}</button></form>")


def install(app: FastAPI, db, settings, outbox: Callable[[str, str, str], None],
            validate_password: Callable[..., List[str]], read_form, session_user) -> None:
    """``read_form(request) -> (fields, files, error_response)``; ``session_user(request)``
    resolves the ``sessionid`` cookie (or any other credential) to a user row."""

    async def fields(request: Request) -> Dict[str, Any]:
        f, _, e = await read_form(request)
        return {} if e else f

    def page(request: Request, title: str, action: str, flds: List[tuple], submit: str,
             errors: Optional[List[str]] = None, status: int = 200):
        tok = csrf_token(request)
        return _with_csrf(_page(title, _form(action, flds, submit, errors, tok), status), request, tok)

    def csrf_failed(request: Request):
        return _page("Forbidden", "<p>CSRF verification failed. Request aborted.</p>", 403)

    # ------------------------------------------------------------------ login / logout
    login_fields = [("username", "Username", "text"), ("password", "Password", "password")]

    @app.get("/login/")
    async def login_page(request: Request):
        return page(request, "Log in", "/login/", login_fields, "Log in")

    @app.post("/login/")
    async def login_submit(request: Request):
        f = await fields(request)
        if not csrf_ok(request, f):
            return csrf_failed(request)
        user = db.find_user(username=str(f.get("username", "")))
        from ..store.db import check_password
        if not user or not check_password(str(f.get("password", "")), user["password"]):
            return page(request, "Log in", "/login/", login_fields, "Log in",
                        ["Please enter a correct username and password."])
        nxt = request.query_params.get("next", "/")
        if not nxt.startswith("/") or nxt.startswith("//"):
            nxt = "/"                                   # no open redirect
        r = RedirectResponse(nxt, status_code=302)
        r.set_cookie(COOKIE, db.token_for(user["id"]), httponly=True, samesite="lax", max_age=SESSION_AGE_S)
        # rotate the CSRF token at login (Django's rotate_token)
        r.set_cookie(CSRF_COOKIE, secrets.token_hex(16), samesite="lax", max_age=365 * 86400)
        return r

    @app.get("/logout/")
    async def logout_confirm(request: Request):
        # a GET never logs out (a cross-site link must not delete the shared API token)
        return page(request, "Log out", "/logout/", [], "Log out")

    @app.post("/logout/")
    async def logout_page(request: Request):
        f = await fields(request)
        if not csrf_ok(request, f):
            return csrf_failed(request)
        u = session_user(request, csrf_verified=True)
        if u:
            db.delete_token(u["id"])
        r = _page("Logged out", "<p>Thanks for spending some quality time with the web site today.</p>")
        r.delete_cookie(COOKIE)
        return r

    # ------------------------------------------------------------------ password change
    change_fields = [("old_password", "Old password", "password"),
                     ("new_password1", "New password", "password"),
                     ("new_password2", "New password confirmation", "password")]

    @app.get("/password_change/")
    async def change_page(request: Request):
        if session_user(request) is None:
            return RedirectResponse("/login/?next=/password_change/", status_code=302)
        return page(request, "Password change", "/password_change/", change_fields, "Change my password")

    @app.post("/password_change/")
    async def change_submit(request: Request):
        f = await fields(request)
        if not csrf_ok(request, f):
            return csrf_failed(request)
        u = session_user(request, csrf_verified=True)
        if u is None:
            return RedirectResponse("/login/?next=/password_change/", status_code=302)
        from ..store.db import check_password
        errs: List[str] = []
        if not check_password(str(f.get("old_password", "")), u["password"]):
            errs.append("Your old password was entered incorrectly.")
        p1, p2 = str(f.get("new_password1", "")), str(f.get("new_password2", ""))
        if p1 != p2:
            errs.append("The two password fields didn't match.")
        errs += validate_password(p1, u["username"], u["email"]) if not errs else []
        if errs:
            return page(request, "Password change", "/password_change/", change_fields, "Change my password", errs)
        db.set_password(u["id"], p1)          # revokes every session; this browser gets a new one
        r = RedirectResponse("/password_change/done/", status_code=302)
        r.set_cookie(COOKIE, db.token_for(u["id"]), httponly=True, samesite="lax", max_age=SESSION_AGE_S)
        return r

    @app.get("/password_change/done/")
    async def change_done(request: Request):
        return _page("Password change successful", "<p>Your password was changed.</p>")

    # ------------------------------------------------------------------ password reset
    @app.get("/password_reset/")
    async def reset_page(request: Request):
        return page(request, "Password reset", "/password_reset/", [("email", "Email", "email")], "Reset my password")

    @app.post("/password_reset/")
    async def reset_submit(request: Request):
        f = await fields(request)
        if not csrf_ok(request, f):
            return csrf_failed(request)
        email = str(f.get("email", ""))
        user = db.find_user(email=email) if email else None
        if user:
            tok = db.new_reset_token(user["id"])
            outbox(email, "Password reset", f"Open /reset/{user['id']}/{tok}/ to choose a new password.")
        return RedirectResponse("/password_reset/done/", status_code=302)   # same answer either way

    @app.get("/password_reset/done/")
    async def reset_done(request: Request):
        return _page("Password reset sent", "<p>We've emailed you instructions for setting your password.</p>")

    set_fields = [("new_password1", "New password", "password"),
                  ("new_password2", "New password confirmation", "password")]

    @app.get("/reset/{uid}/{token}/")
    async def reset_confirm_page(uid: int, token: str, request: Request):
        return page(request, "Enter new password", f"/reset/{uid}/{token}/", set_fields, "Change my password")

    @app.post("/reset/{uid}/{token}/")
    async def reset_confirm_submit(uid: int, token: str, request: Request):
        f = await fields(request)
        if not csrf_ok(request, f):
            return csrf_failed(request)
        user = db.get_user(uid)
        p1, p2 = str(f.get("new_password1", "")), str(f.get("new_password2", ""))
        errs: List[str] = []
        if p1 != p2:
            errs.append("The two password fields didn't match.")
        elif user is not None:
            errs += validate_password(p1, user["username"], user["email"])
        if errs:
            return page(request, "Enter new password", f"/reset/{uid}/{token}/", set_fields, "Change my password",
                        errs)
        if user is None or not db.use_reset_token(uid, token):
            return _page("Password reset unsuccessful", "<p>The password reset link was invalid.</p>", 400)
        db.set_password(uid, p1)
        return RedirectResponse("/reset/done/", status_code=302)

    @app.get("/reset/done/")
    async def reset_complete(request: Request):
        return _page("Password reset complete", "<p>Your password has been set. <a href='/login/'>Log in</a></p>")

    # ------------------------------------------------------------------ admin index
    @app.get("/admin/")
    async def admin_index(request: Request):
        u = session_user(request)
        if u is None or not u.get("is_staff"):
            return RedirectResponse("/login/?next=/admin/", status_code=302)
        rows = "".join(f"<tr><td>{html.escape(t)}</td><td>{n}</td></tr>" for t, n in db.table_counts())
        return _page("Site administration",
                     f"<p>Welcome, {html.escape(u['username'])}.</p>"
                     f"<table><tr><th>table</th><th>rows</th></tr>{rows}</table>")

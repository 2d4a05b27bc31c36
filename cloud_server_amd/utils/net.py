"""Outbound HTTP(S) fetch for URL datasets, with an SSRF guard.

Reference: ``handle_url_local`` (apps/data/views.py:193-208) calls
``urllib.request.urlretrieve`` on whatever the user posted.  Here:

* only ``http`` and ``https`` URLs are fetched (``file://``, ``ftp://`` and the rest are
  refused: a ``file://`` URL would copy a server file — the database, the outbox — into
  the caller's dataset);
* the destination must be a public address: loopback, private, link-local, multicast,
  reserved and unspecified addresses are refused unless the deployment opts in
  (``CSA_URL_ALLOW_PRIVATE=1``, used by tests that serve fixtures on 127.0.0.1).  The
  check runs on the address the socket actually CONNECTED to (``getpeername``), so DNS
  rebinding and redirects to an internal host are caught at every hop;
* a size cap bounds every download.
"""
from __future__ import annotations

import http.client
import ipaddress
import os
import urllib.parse
import urllib.request
from typing import Optional

ALLOWED_SCHEMES = ("http", "https")


class FetchRefused(ValueError):
    pass


def address_allowed(addr: str, allow_private: bool) -> bool:
    try:
        ip = ipaddress.ip_address(addr.split("%", 1)[0])
    except ValueError:
        return False
    if allow_private:
        return not ip.is_unspecified and not ip.is_multicast
    if isinstance(ip, ipaddress.IPv6Address) and ip.ipv4_mapped is not None:
        ip = ip.ipv4_mapped
    return ip.is_global and not (ip.is_multicast or ip.is_reserved or ip.is_link_local
                                 or ip.is_loopback or ip.is_private or ip.is_unspecified)


def _checked(conn_cls, allow_private: bool):
    class Conn(conn_cls):
        def connect(self):
            super().connect()
            peer = self.sock.getpeername()[0]
            if not address_allowed(peer, allow_private):
                self.sock.close()
                raise FetchRefused(f"destination address {peer} is not allowed")
    return Conn


def _opener(allow_private: bool) -> urllib.request.OpenerDirector:
    HC = _checked(http.client.HTTPConnection, allow_private)
    HSC = _checked(http.client.HTTPSConnection, allow_private)

    class H(urllib.request.HTTPHandler):
        def http_open(self, req):
            return self.do_open(HC, req)

    class HS(urllib.request.HTTPSHandler):
        def https_open(self, req):
            return self.do_open(HSC, req, context=self._context)

    class Redirect(urllib.request.HTTPRedirectHandler):
        def redirect_request(self, req, fp, code, msg, headers, newurl):
            if urllib.parse.urlsplit(newurl).scheme.lower() not in ALLOWED_SCHEMES:
                raise FetchRefused(f"redirect to a non-http(s) URL refused: {newurl}")
            return super().redirect_request(req, fp, code, msg, headers, newurl)

    # build_opener would add the default handlers (FileHandler, FTPHandler, ...): build
    # the director by hand so only http(s) can ever be opened
    od = urllib.request.OpenerDirector()
    for h in (H(), HS(), Redirect(), urllib.request.HTTPErrorProcessor(),
              urllib.request.HTTPDefaultErrorHandler()):
        od.add_handler(h)
    return od


def check_url(url: str) -> str:
    parts = urllib.parse.urlsplit(url)
    if parts.scheme.lower() not in ALLOWED_SCHEMES or not parts.hostname:
        raise FetchRefused(f"only http(s) URLs are fetched: {url!r}")
    return url


def fetch(url: str, dest_path: str, allow_private: Optional[bool] = None, timeout: float = 60.0,
          max_bytes: int = 1 << 30) -> int:
    """Download ``url`` to ``dest_path``; returns the byte count.  Raises FetchRefused for
    a refused scheme/address/size, OSError for network failures."""
    if allow_private is None:
        allow_private = os.environ.get("CSA_URL_ALLOW_PRIVATE", "0") == "1"
    check_url(url)
    n = 0
    tmp = dest_path + ".part"
    try:
        with _opener(allow_private).open(url, timeout=timeout) as r, open(tmp, "wb") as out:
            while True:
                chunk = r.read(1 << 20)
                if not chunk:
                    break
                n += len(chunk)
                if n > max_bytes:
                    raise FetchRefused(f"download exceeds {max_bytes} bytes")
                out.write(chunk)
        os.replace(tmp, dest_path)
    finally:
        if os.path.exists(tmp):
            os.remove(tmp)
    return n


__all__ = ["FetchRefused", "address_allowed", "check_url", "fetch"]

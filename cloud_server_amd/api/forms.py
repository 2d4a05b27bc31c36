"""Request-body parsing: multipart/form-data, urlencoded forms and JSON.

The reference read uploads through Django's ``request.POST`` / ``request.FILES``
(apps/data/views.py:41, 96-98).  Starlette's form parser needs the ``python-multipart``
package, which is not installed here, so multipart is parsed directly (RFC 7578):
split on the boundary, parse each part's headers, keep file parts as bytes.
"""
from __future__ import annotations

import json
import re
from dataclasses import dataclass
from typing import Any, Dict, Optional, Tuple
from urllib.parse import parse_qs


@dataclass
class UploadFile:
    filename: str
    content_type: str
    data: bytes


class FormError(ValueError):
    pass


_PARAM = re.compile(r';\s*([a-zA-Z0-9_*-]+)\s*=\s*("(?:[^"\\]|\\.)*"|[^;]*)')


def _header_params(value: str) -> Tuple[str, Dict[str, str]]:
    main = value.split(";", 1)[0].strip().lower()
    params: Dict[str, str] = {}
    for k, v in _PARAM.findall(value):
        v = v.strip()
        if v.startswith('"') and v.endswith('"'):
            v = v[1:-1].replace('\\"', '"').replace("\\\\", "\\")
        params[k.lower()] = v
    return main, params


def parse_multipart(body: bytes, content_type: str) -> Tuple[Dict[str, str], Dict[str, UploadFile]]:
    _, params = _header_params(content_type)
    boundary = params.get("boundary")
    if not boundary:
        raise FormError("multipart body without boundary")
    delim = b"--" + boundary.encode("latin-1")
    fields: Dict[str, str] = {}
    files: Dict[str, UploadFile] = {}
    for chunk in body.split(delim)[1:]:
        if chunk.startswith(b"--"):
            break
        if chunk.startswith(b"\r\n"):
            chunk = chunk[2:]
        if chunk.endswith(b"\r\n"):
            chunk = chunk[:-2]
        head, sep, data = chunk.partition(b"\r\n\r\n")
        if not sep:
            continue
        headers: Dict[str, str] = {}
        for line in head.decode("utf-8", "replace").split("\r\n"):
            if ":" in line:
                k, v = line.split(":", 1)
                headers[k.strip().lower()] = v.strip()
        disp, dparams = _header_params(headers.get("content-disposition", ""))
        name = dparams.get("name")
        if disp != "form-data" or name is None:
            continue
        fname = dparams.get("filename*") or dparams.get("filename")
        if fname is not None:
            if fname.lower().startswith("utf-8''"):
                from urllib.parse import unquote
                fname = unquote(fname[7:])
            files[name] = UploadFile(fname, headers.get("content-type", "application/octet-stream"), data)
        else:
            fields[name] = data.decode("utf-8", "replace")
    return fields, files


async def read_form(request, max_bytes: int) -> Tuple[Dict[str, Any], Dict[str, UploadFile]]:
    """Fields + files of a request, whatever its encoding (multipart, urlencoded, JSON)."""
    body = await request.body()
    if len(body) > max_bytes:
        raise FormError("request body too large")
    ct = request.headers.get("content-type", "")
    kind = ct.split(";", 1)[0].strip().lower()
    if kind == "multipart/form-data":
        return parse_multipart(body, ct)
    if kind == "application/x-www-form-urlencoded":
        q = parse_qs(body.decode("utf-8", "replace"), keep_blank_values=True)
        return {k: v[-1] for k, v in q.items()}, {}
    if body.strip():
        try:
            obj = json.loads(body)
        except json.JSONDecodeError:
            raise FormError("body is not valid JSON")
        if isinstance(obj, dict):
            return obj, {}
        raise FormError("JSON body must be an object")
    return {}, {}


def encode_multipart(fields: Dict[str, str], files: Dict[str, Tuple[str, bytes, str]],
                     boundary: str = "----csaBoundary7d9f") -> Tuple[bytes, str]:
    """Client-side helper (tests / CLI): build a multipart body."""
    out = []
    for k, v in fields.items():
        out.append(f"--{boundary}\r\nContent-Disposition: form-data; name=\"{k}\"\r\n\r\n".encode() +
                   str(v).encode() + b"\r\n")
    for k, (fname, data, ctype) in files.items():
        out.append(f"--{boundary}\r\nContent-Disposition: form-data; name=\"{k}\"; filename=\"{fname}\"\r\n"
                   f"Content-Type: {ctype}\r\n\r\n".encode() + data + b"\r\n")
    out.append(f"--{boundary}--\r\n".encode())
    return b"".join(out), f"multipart/form-data; boundary={boundary}"

"""The website's node-side server (the reference's Website/Website/server.js, metrics/metricService.js,
util/localCache.js, auth.js and web.composition.json), served by the control plane's FastAPI app:

* ``/`` and every enabled page route of ``web.composition.json`` (``/home``, ``/config*``, ``/dashboard*``,
  ``/jobs*``) return the single-page shell (server.js:86-101); the client router picks the package module;
* ``/dist/<path>`` serves the ES-module packages under ``dxa/service/webui`` (dist.js: static files);
* ``/api/web-composition`` (server.js:104-107), ``/api/enableLocalOneBox`` (:110-114), ``/api/user`` (the identity
  the datax-common ``user`` module reads, auth.js), ``/api/functionenabled`` (the role-gated UI switches of
  web.composition.json ``functionsEnabled``), ``/api/metrics/<name>/freshness`` (metricService.js:14,93).

The page packages mirror Website/Packages: ``common`` (datax-common), ``home`` (datax-home), ``pipeline``
(datax-pipeline: flow list + flow definition), ``query`` (datax-query LiveQuery), ``metrics`` (datax-metrics) and
``jobs`` (datax-jobs). They are plain ES modules: no bundler, no external assets (deployments have no network).
"""
from __future__ import annotations

import json
import mimetypes
import os
from typing import Any, Dict, Optional

from fastapi import FastAPI, Header, HTTPException, Request
from fastapi.responses import FileResponse, HTMLResponse, JSONResponse

WEBUI_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "webui")

_MIME = {".js": "text/javascript", ".css": "text/css", ".json": "application/json", ".html": "text/html",
         ".svg": "image/svg+xml"}


def composition() -> Dict[str, Any]:
    with open(os.path.join(WEBUI_DIR, "web.composition.json")) as f:
        return json.load(f)


def page_routes(comp: Optional[Dict[str, Any]] = None):
    """server.js:92-101 — the route paths of the enabled, non-external pages (``:param`` segments kept)."""
    comp = comp or composition()
    out = []
    for p in comp["client"]["pages"]:
        if p.get("enable") and not p.get("externalUrl"):
            out.append((p["routePath"], bool(p.get("supportSubRoute"))))
    return out


def enabled_functions(comp: Dict[str, Any], is_writer: bool, onebox: bool):
    """The UI switches a user gets: every ``enabledForWriter`` switch for writers (readers get none), minus the
    ``disabledForLocalOneBox`` ones in onebox mode (datax-common functionEnabled)."""
    fe = comp.get("functionsEnabled", {})
    names = list(dict.fromkeys(fe.get("enabledForWriter", []))) if is_writer else []
    if onebox:
        off = set(fe.get("disabledForLocalOneBox", []))
        names = [n for n in names if n not in off]
    return {n: True for n in names}


def _static_path(rel: str) -> str:
    root = os.path.realpath(WEBUI_DIR)
    path = os.path.realpath(os.path.join(root, rel))
    if not path.startswith(root + os.sep) or not os.path.isfile(path):
        raise HTTPException(status_code=404, detail=f"no such file {rel}")
    return path


def mount_website(app: FastAPI, st, authn, onebox: Optional[bool] = None):
    """Register the website routes on the control-plane app. ``onebox`` defaults to the authenticator's local mode
    (enableLocalOneBox in the reference's config.js)."""
    if onebox is None:
        onebox = authn.mode in ("local", "off")
    comp = composition()

    def index():
        with open(os.path.join(WEBUI_DIR, "index.html")) as f:
            return HTMLResponse(f.read())

    @app.get("/", response_class=HTMLResponse)
    def home():
        return index()

    for path, sub in page_routes(comp):
        pattern = path
        # FastAPI path syntax: '/config/edit/:id' -> '/config/edit/{id}'; sub-routes take any suffix
        pattern = "/".join("{" + seg[1:] + "}" if seg.startswith(":") else seg for seg in pattern.split("/"))
        app.add_api_route(pattern, index, methods=["GET"], response_class=HTMLResponse, include_in_schema=False)
        if sub:
            app.add_api_route(pattern.rstrip("/") + "/{rest:path}", index, methods=["GET"],
                              response_class=HTMLResponse, include_in_schema=False)

    @app.get("/dist/{rel:path}")
    def dist(rel: str):
        path = _static_path(rel)
        ext = os.path.splitext(path)[1]
        return FileResponse(path, media_type=_MIME.get(ext) or mimetypes.guess_type(path)[0] or "text/plain",
                            headers={"Cache-Control": "no-cache"})

    @app.get("/api/web-composition")
    def web_composition():
        return JSONResponse(comp["client"])

    @app.get("/api/enableLocalOneBox")
    def enable_local_onebox():
        return {"enableLocalOneBox": bool(onebox)}

    def _identity(request: Request, authorization: Optional[str], roles: Optional[str]):
        from .auth import AuthError
        host = request.client.host if request.client else None
        try:
            claims = authn.check(False, authorization, roles, host)
        except AuthError as e:
            raise HTTPException(status_code=e.status, detail=str(e))
        try:
            authn.check(True, authorization, roles, host)
            writer = True
        except AuthError:
            writer = False
        name = claims.get("name") or claims.get("preferred_username") or claims.get("upn") or \
            ("local user" if authn.mode in ("local", "off") else claims.get("oid", ""))
        rl = claims.get("roles") or []
        rl = [rl] if isinstance(rl, str) else list(rl)
        if authn.mode in ("local", "off"):
            rl = ["DataXWriter"]
        return {"id": claims.get("oid") or claims.get("sub") or "local", "name": name, "roles": rl,
                "isWriter": writer, "authMode": authn.mode}

    @app.get("/api/user")
    def user(request: Request, authorization: Optional[str] = Header(None),
             x_dxa_roles: Optional[str] = Header(None)):
        return _identity(request, authorization, x_dxa_roles)

    @app.get("/api/functionenabled")
    def function_enabled(request: Request, authorization: Optional[str] = Header(None),
                         x_dxa_roles: Optional[str] = Header(None)):
        ident = _identity(request, authorization, x_dxa_roles)
        return enabled_functions(comp, ident["isWriter"], bool(onebox))

    @app.get("/api/metrics/{name}/freshness")
    def freshness(name: str, request: Request, authorization: Optional[str] = Header(None),
                  x_dxa_roles: Optional[str] = Header(None)):
        """metricService.js:93 — the newest point of a metric (the dashboard's data-freshness box).  Reader role."""
        _identity(request, authorization, x_dxa_roles)
        rows = st.metrics.zrangebyscore(name, float("-inf"), float("inf"))
        return [json.loads(v) for _, v in rows[-1:]]

"""foremast-service REST API on :8099 (foremast-service/cmd/manager/main.go:300-351).

Routes (identical paths, verbs and JSON):
  POST /v1/healthcheck/create                -> {"jobId", "statusCode": 200, "status": "new"}
  GET  /v1/healthcheck/id/{id}               -> job status (+ last 10 hpalogs, + anomaly map)
  GET  /alert/{appName}/{namespace}/{strategy} -> HPA logs of ``app:ns:strategy``
  GET  /api/v1/{queryproxy}                  -> CORS proxy to <QUERY_SERVICE_ENDPOINT>api/v1/query_range
Extra (not in the reference):
  GET  /healthz, GET /v1/healthcheck/jobs (list), POST /v1/healthcheck/abort/{id} (client abort,
  the "abort by client" edge of the state diagram), GET /metrics (Prometheus exposition of the
  embedded brain's registry when one is attached).
"""
from __future__ import annotations

import logging

import httpx
from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, PlainTextResponse, Response

from ..api import jobs as J
from ..api import status as ST
from ..api.models import ApplicationHealthAnalyzeRequest
from ..config import ServiceConfig
from .store import JobStore, MemoryStore

log = logging.getLogger("foremast.service")


def _err(code: int, msg: str) -> JSONResponse:
    return JSONResponse({"error": msg}, status_code=code)


def create_app(store: JobStore | None = None, cfg: ServiceConfig | None = None, registry=None,
               http_client: httpx.AsyncClient | None = None) -> FastAPI:
    cfg = cfg or ServiceConfig()
    store = store or MemoryStore()
    app = FastAPI(title="foremast-service (MI355X)", version="1.0")
    app.state.store = store
    app.state.cfg = cfg

    @app.post("/v1/healthcheck/create")
    async def register_entry(request: Request):
        try:
            body = await request.json()
            if not isinstance(body, dict):
                raise ValueError("not an object")
            req = ApplicationHealthAnalyzeRequest.from_dict(body)
        except Exception as e:  # BindJSON failure (main.go:153-156)
            log.info("bad request: %s", e)
            return _err(400, "Bad request")
        try:
            doc = J.build_document(req)
        except J.RequestError as e:
            return _err(e.code, e.msg)
        try:
            job_id, _ = store.create(doc)
        except Exception as e:  # CreateNewDoc failure -> 500
            return _err(500, str(e))
        return JSONResponse(J.new_response(job_id, 0, "new"))

    @app.get("/v1/healthcheck/id/{job_id}")
    async def search_by_id(job_id: str):
        try:
            doc = store.get(job_id)
        except Exception as e:
            return JSONResponse({"jobId": job_id, "statusCode": 500, "status": "unknown", "reason": str(e)},
                                status_code=500)
        if doc is None:
            return JSONResponse({"jobId": job_id, "statusCode": 404, "status": "unknown", "reason": "Job not found"},
                                status_code=404)
        try:
            logs = store.hpalogs(job_id, 10)
        except Exception as e:
            doc.status_code, doc.reason = "500", str(e)
            return JSONResponse(J.to_response(doc, None), status_code=500)
        if not logs:
            doc.reason = "Job HPA log not found" if not doc.reason else doc.reason
            return JSONResponse(J.to_response(doc, None))
        return JSONResponse(J.to_response(doc, logs))

    @app.get("/alert/{app_name}/{namespace}/{strategy}")
    async def hpa_alert(app_name: str, namespace: str, strategy: str):
        jid = f"{app_name}:{namespace}:{strategy}"
        try:
            logs = store.hpalogs(jid, 10)
        except Exception as e:
            return JSONResponse(J.hpa_alert_response(jid, [], 500, str(e)), status_code=500)
        if not logs:
            return JSONResponse(J.hpa_alert_response(jid, [], 404, "HPA log not found"), status_code=404)
        return JSONResponse(J.hpa_alert_response(jid, logs, 200))

    @app.get("/api/v1/{queryproxy}")
    async def query_proxy(queryproxy: str, request: Request):
        target = cfg.query_endpoint + "api/v1/query_range?" + request.url.query
        headers = {"Access-Control-Allow-Origin": "*"}
        try:
            client = http_client or httpx.AsyncClient(timeout=90.0)
            r = await client.get(target)
            if http_client is None:
                await client.aclose()
        except Exception:
            return JSONResponse({"error": "invoke query " + target + " failed "}, status_code=400, headers=headers)
        # the reference returns the upstream body as a JSON *string* (context.JSON(200, string(contents)))
        return JSONResponse(r.text, headers=headers)

    @app.post("/v1/healthcheck/abort/{job_id}")
    async def abort(job_id: str):
        d = store.update(job_id, status=ST.ABORT, reason="aborted by client")
        if d is None:
            return JSONResponse({"jobId": job_id, "statusCode": 404, "status": "unknown", "reason": "Job not found"},
                                status_code=404)
        return JSONResponse(J.new_response(job_id, 200, ST.to_external(d.status)))

    @app.get("/v1/healthcheck/jobs")
    async def list_jobs(status: str | None = None):
        out = [{"jobId": d.id, "appName": d.app_name, "strategy": d.strategy, "status": d.status,
                "external": ST.to_external(d.status), "modified_at": d.modified_at}
               for d in store.all_docs() if status is None or d.status == status]
        return JSONResponse(out)

    # ------------------------------------------------------------ dashboard (R19)
    async def _prom_range(q: str, start: int, end: int, step: int) -> dict:
        import urllib.parse
        url = cfg.query_endpoint + "api/v1/query_range?" + urllib.parse.urlencode(
            {"query": q, "start": start, "end": end, "step": step})
        try:
            client = http_client or httpx.AsyncClient(timeout=30.0)
            r = await client.get(url)
            if http_client is None:
                await client.aclose()
            return r.json()
        except Exception:
            return {}

    @app.get("/dashboard/api/{namespace}/{app_name}")
    async def dashboard_api(namespace: str, app_name: str, minutes: int = 15):
        from ..dashboard.data import dashboard_data_async
        return JSONResponse(await dashboard_data_async(_prom_range, namespace, app_name, minutes=minutes))

    @app.get("/dashboard/{namespace}/{app_name}")
    async def dashboard_page(namespace: str, app_name: str):
        from fastapi.responses import HTMLResponse
        from ..dashboard.page import render
        return HTMLResponse(render(namespace, app_name))

    @app.get("/healthz")
    async def healthz():
        return PlainTextResponse("ok")

    @app.get("/metrics")
    async def metrics():
        if registry is None:
            return PlainTextResponse("", status_code=404)
        from prometheus_client import CONTENT_TYPE_LATEST, generate_latest
        return Response(generate_latest(registry), media_type=CONTENT_TYPE_LATEST)

    return app


def app_from_env() -> FastAPI:
    """Factory for multi-worker uvicorn (each worker opens the store itself)."""
    from .store import open_store
    cfg = ServiceConfig.from_env()
    return create_app(open_store(cfg.store, cfg.elastic_url), cfg)


def main() -> None:  # pragma: no cover - entry point
    import argparse
    import os

    import uvicorn

    ap = argparse.ArgumentParser(description="foremast-service (MI355X framework)")
    ap.add_argument("--port", type=int, default=None)
    ap.add_argument("--store", default=None, help="memory | sqlite:<path> | elasticsearch")
    ap.add_argument("--workers", type=int, default=int(os.environ.get("SERVICE_WORKERS", "1")),
                    help="uvicorn worker processes (sqlite/elasticsearch stores only: memory is per process)")
    a = ap.parse_args()
    cfg = ServiceConfig.from_env()
    if a.store:
        cfg.store = a.store
        os.environ["FOREMAST_STORE"] = a.store
    port = a.port or cfg.port
    if a.workers > 1 and cfg.store != "memory":
        uvicorn.run("foremast_amd.service.app:app_from_env", factory=True, host="0.0.0.0", port=port,
                    workers=a.workers, log_level="warning", access_log=False)
        return
    from .store import open_store
    uvicorn.run(create_app(open_store(cfg.store, cfg.elastic_url), cfg), host="0.0.0.0", port=port,
                log_level="warning", access_log=False)


if __name__ == "__main__":  # pragma: no cover
    main()

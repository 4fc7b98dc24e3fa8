"""``python -m foremast_amd.cli <command>`` — one entry point for every
process of the framework plus the operator-facing commands.

  service     REST service (:8099)                 foremast-service/cmd/manager/main.go
  brain       scoring engine, one rank per GPU      (foremast-brain, external in the reference)
  barrelman   K8s controller                        foremast-barrelman/cmd/manager/main.go
  trigger     Wavefront batch scanner               foremast-trigger/cmd/manager/main.go
  watch APP   start continuous monitoring           bin/kubectl-watch
  unwatch APP stop continuous monitoring            bin/kubectl-unwatch
  status APP  phase / job / anomaly of a DeploymentMonitor
  manifests   write the deploy bundle
  validate F  check DeploymentMonitor/DeploymentMetadata YAML against the CRD schema
  demo        fault-injection demo workload (examples/spring-boot-demo analogue)
  sidecar     metrics reverse-proxy sidecar: foremast-metrics series for any app (JVM included)
"""
from __future__ import annotations

import argparse
import json
import os
import sys


def set_continuous(kube, namespace: str, app: str, on: bool) -> dict:
    """What ``kubectl watch/unwatch`` does: merge-patch ``spec.continuous``
    of the app's DeploymentMonitor (the MonitorController reacts to the flip)."""
    from .controller import kube as K
    return kube.patch_merge(K.MONITORS, namespace, app, {"spec": {"continuous": bool(on)}})


def monitor_status(kube, namespace: str, app: str) -> dict:
    from .api import crd
    from .controller import kube as K
    m = crd.DeploymentMonitor.from_dict(kube.get(K.MONITORS, namespace, app))
    st = m.status
    return {"name": m.name, "namespace": m.namespace, "phase": st.phase, "jobId": st.job_id,
            "continuous": m.spec.continuous, "remediationTaken": st.remediation_taken,
            "anomalousMetrics": [a.name for a in st.anomaly.anomalous_metrics],
            "hpaScoreEnabled": st.hpa_score_enabled, "hpaLogs": len(st.hpa_logs or [])}


def validate_docs(docs: list[dict]) -> list[str]:
    from .api import crd
    from .deploy.manifests import openapi_schema, validate
    import typing
    errs = []
    kinds = {"DeploymentMonitor": crd.DeploymentMonitor, "DeploymentMetadata": crd.DeploymentMetadata}
    for i, d in enumerate(docs):
        cls = kinds.get((d or {}).get("kind", ""))
        if cls is None:
            continue
        hints = typing.get_type_hints(cls)
        for part in ("spec", "status"):
            if part in d:
                errs += [f"doc {i} {e}" for e in validate(d[part], openapi_schema(hints[part]), f"$.{part}")]
    return errs


def _kube(a):
    from .controller.kube import HttpKube
    return HttpKube(a.apiserver, a.token)


def brain_main(argv=None) -> None:  # pragma: no cover - process entry
    import torch
    from .config import BrainConfig
    from .engine.brain import Brain
    from .engine.exporter import BrainExporter
    from .parallel import dist as D
    from .service.store import open_store
    ap = argparse.ArgumentParser(prog="foremast brain")
    ap.add_argument("--store", default=os.environ.get("FOREMAST_STORE", "memory"))
    ap.add_argument("--elastic-url", default=os.environ.get("ELASTIC_URL", ""))
    ap.add_argument("--batch", type=int, default=int(os.environ.get("BRAIN_BATCH", "4096")))
    a = ap.parse_args(argv)
    info = D.env_info()
    dev = torch.device("cuda", info.local_rank) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    info = D.init_distributed(device=dev)
    if info.world > 1 and dev.type == "cuda" and os.environ.get("BRAIN_XGMI_BOARD", "1") != "0":
        # gauge vectors and verdict rows between the ranks over xGMI (HIP IPC
        # board on rank 0, self-tested); the TCPStore mailbox otherwise
        from .parallel import board
        b = board.setup(dev)
        print(f"rank {info.rank}: rank exchange over "
              f"{'the xGMI board' if b is not None else 'the TCPStore mailbox'}", file=sys.stderr, flush=True)
    cfg = BrainConfig.from_env()
    exporter = BrainExporter()
    if info.is_main:
        exporter.serve(cfg.metrics_port)
    brain = Brain(open_store(a.store, a.elastic_url), cfg, device=dev, exporter=exporter, batch_size=a.batch,
                  worker_id=f"{os.uname().nodename}-rank{info.rank}")
    ckpt = os.environ.get("BRAIN_CHECKPOINT_DIR")
    if ckpt:
        brain.load_checkpoint(ckpt)
        n = brain.load_history(ckpt)                  # warm restart: resident history without a re-fetch
        print(f"restored {n} resident history rows from {ckpt}", file=sys.stderr, flush=True)
    # SIGTERM (pod shutdown; torchrun forwards it to every rank) ends the
    # loop after the current cycle and writes a final checkpoint
    import signal
    import threading
    stop = threading.Event()
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, lambda *_: stop.set())
    brain.run_forever(stop=stop, checkpoint_dir=ckpt or None,
                      checkpoint_every=int(os.environ.get("BRAIN_CHECKPOINT_EVERY", "30")))


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] in ("-h", "--help"):
        print(__doc__)
        return 0
    cmd, rest = argv[0], argv[1:]
    from .utils import logs
    logs.setup(component=cmd)
    if cmd == "service":
        from .service import app
        sys.argv = ["foremast service"] + rest
        app.main()
        return 0
    if cmd == "brain":
        brain_main(rest)
        return 0
    if cmd == "barrelman":
        from .controller import manager
        sys.argv = ["foremast barrelman"] + rest
        manager.main()
        return 0
    if cmd == "trigger":
        from .trigger import trigger
        trigger.main()
        return 0
    if cmd == "sidecar":
        from .emitter import sidecar
        sidecar.main(rest)
        return 0
    if cmd == "demo":
        from .demo import app as demo
        sys.argv = ["foremast demo"] + rest
        demo.main()
        return 0
    if cmd == "manifests":
        from .deploy.manifests import write
        mp = argparse.ArgumentParser(prog="foremast manifests", description="write the deploy bundle")
        mp.add_argument("out_dir", nargs="?", default="deploy/foremast")
        for p in write(mp.parse_args(rest).out_dir):
            print(p)
        return 0
    if cmd == "validate":
        import yaml
        vp = argparse.ArgumentParser(prog="foremast validate",
                                     description="check DeploymentMonitor / DeploymentMetadata YAML against the CRD schema")
        vp.add_argument("files", nargs="+")
        docs = [d for f in vp.parse_args(rest).files for d in yaml.safe_load_all(open(f))]
        errs = validate_docs(docs)
        for e in errs:
            print(e)
        return 1 if errs else 0
    ap = argparse.ArgumentParser(prog=f"foremast {cmd}")
    ap.add_argument("app")
    ap.add_argument("-n", "--namespace", default="default")
    ap.add_argument("--apiserver", default=None)
    ap.add_argument("--token", default=None)
    a = ap.parse_args(rest)
    if cmd in ("watch", "unwatch"):
        set_continuous(_kube(a), a.namespace, a.app, cmd == "watch")
        print(f"Foremast {'starts' if cmd == 'watch' else 'stops'} watching application {a.app}")
        return 0
    if cmd == "status":
        print(json.dumps(monitor_status(_kube(a), a.namespace, a.app), indent=2))
        return 0
    print(f"unknown command {cmd!r}\n{__doc__}", file=sys.stderr)
    return 2


if __name__ == "__main__":  # pragma: no cover
    sys.exit(main())

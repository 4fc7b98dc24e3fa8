"""Barrelman process wiring (foremast-barrelman/cmd/manager/main.go:35-111):
informers for Deployments (30 s resync), DeploymentMonitors (10 s) and HPAs,
the 10 s status poller, and N deployment workers."""
from __future__ import annotations

import logging
import threading
import time

from ..config import BarrelmanConfig
from . import kube as K
from .barrelman import Barrelman, Dispatcher
from .controllers import DeploymentController, HpaController, MonitorController

log = logging.getLogger("foremast.manager")


class Manager:
    def __init__(self, kube: K.KubeAPI, cfg: BarrelmanConfig | None = None, analyst_factory=None, clock=time.time,
                 sleep=time.sleep, inline: bool = False):
        self.kube = kube
        self.cfg = cfg or BarrelmanConfig()
        self.barrelman = Barrelman(kube, self.cfg, analyst_factory, clock, sleep, Dispatcher(inline=inline))
        self.deployments = DeploymentController(kube, self.barrelman, clock)
        self.monitors = MonitorController(kube, self.barrelman, clock)
        self.hpas = HpaController(kube, self.barrelman, clock)

    def register_watches(self) -> None:
        self.kube.watch(K.DEPLOYMENTS, self.deployments.handle, 30.0)
        self.kube.watch(K.MONITORS, self.monitors.handle, 10.0)
        self.kube.watch(K.HPAS, self.hpas.handle, 30.0)

    def run(self, stop: threading.Event) -> None:  # pragma: no cover - process loop
        self.register_watches()
        self.barrelman.start_poller(stop)
        self.deployments.run_workers(self.cfg.workers, stop)
        stop.wait()


def main() -> None:  # pragma: no cover - entry point
    import argparse
    import signal
    ap = argparse.ArgumentParser(description="foremast barrelman controller (MI355X framework)")
    ap.add_argument("--apiserver", default=None, help="API server URL (default: in-cluster)")
    ap.add_argument("--token", default=None)
    a = ap.parse_args()
    from ..utils import logs
    logs.setup(component="barrelman")
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    signal.signal(signal.SIGINT, lambda *_: stop.set())
    Manager(K.HttpKube(a.apiserver, a.token), BarrelmanConfig.from_env()).run(stop)


if __name__ == "__main__":  # pragma: no cover
    main()

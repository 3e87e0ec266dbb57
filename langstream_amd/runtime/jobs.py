"""Entry points of the setup and deployer Jobs the operator runs per application revision.

Parity: RT/application/ApplicationSetupRunner.java:30-139 (``application-setup``: topics
and assets -- ``ApplicationDeployer.setup`` -- or, in the cleanup phase, deletion of the
topics / assets whose deletion-mode is ``delete``) and RT/deployer/RuntimeDeployer.java
(``deployer-runtime``: the Agent CRs + config Secrets of the plan, or their deletion).

  python -m langstream_amd.runtime.jobs application-setup /app-config/config
  python -m langstream_amd.runtime.jobs deployer-runtime  /app-config/config

The config file is the JSON the operator writes into ``langstream-runtime-config-<app>``
(applicationId, namespace, tenant, application files + instance, secrets, codeArchiveId,
image); the phase comes from ``LANGSTREAM_JOB_PHASE`` (setup | cleanup, deploy | delete).
The deployer talks to the API server in-cluster (service account), or to
``$LANGSTREAM_KUBE_API`` when set.
"""
from __future__ import annotations

import json
import logging
import os
import sys
from typing import List, Optional

log = logging.getLogger(__name__)


def _load(path: str) -> dict:
    with open(path, encoding="utf-8") as f:
        return json.load(f)


def _plan(cfg: dict):
    from ..core.deployer import ApplicationDeployer
    from ..core.parser import build_application_instance
    files = cfg.get("application") or {}
    built = build_application_instance(files.get("files") or {}, files.get("instance"), cfg.get("secrets"))
    app = getattr(built, "application", built)
    dep = ApplicationDeployer()
    return dep, dep.create_implementation(cfg["applicationId"], app), cfg.get("tenant") or "default"


def application_setup(cfg: dict, phase: str) -> None:
    dep, plan, tenant = _plan(cfg)
    if phase == "cleanup":
        dep.cleanup(tenant, plan)
    else:
        dep.setup(tenant, plan)
    log.info("application-setup %s of %s done", phase, cfg["applicationId"])


def deployer_runtime(cfg: dict, phase: str) -> None:
    from ..operator import delete_agents, deploy_agents
    from ..operator.kube import CR_API, KubeClient
    kube = KubeClient(os.environ.get("LANGSTREAM_KUBE_API") or None, os.environ.get("LANGSTREAM_KUBE_TOKEN"))
    ns, name = cfg["namespace"], cfg["applicationId"]
    if phase == "delete":
        delete_agents(kube, ns, name)
    else:
        app_cr = kube.get(CR_API, "Application", ns, name)
        if app_cr is None:
            raise RuntimeError(f"Application {ns}/{name} not found")
        _, plan, tenant = _plan(cfg)
        deploy_agents(kube, app_cr, plan, tenant, cfg.get("image") or "langstream-amd/runtime:latest")
    log.info("deployer-runtime %s of %s done", phase, name)


def main(argv: Optional[List[str]] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(message)s")
    if len(argv) != 2 or argv[0] not in ("application-setup", "deployer-runtime"):
        print("usage: python -m langstream_amd.runtime.jobs {application-setup|deployer-runtime} CONFIG",
              file=sys.stderr)
        return 2
    cfg = _load(argv[1])
    phase = os.environ.get("LANGSTREAM_JOB_PHASE", "")
    if argv[0] == "application-setup":
        application_setup(cfg, phase or "setup")
    else:
        deployer_runtime(cfg, phase or "deploy")
    return 0


if __name__ == "__main__":
    sys.exit(main())

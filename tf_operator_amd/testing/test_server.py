"""Fault-injection replica used by the E2E suites (reference:
test/test-server/test_app.py:19-82).

GET /            hello world
GET /tfconfig    the TF_CONFIG env var verbatim
GET /runconfig   the tf.estimator RunConfig fields derived from TF_CONFIG
                 (computed here without TensorFlow: task_type, task_id,
                 cluster_spec, is_chief, master, num_worker_replicas,
                 num_ps_replicas -- what estimator_runconfig_tests.py:25-97 checks)
GET /env         the RCCL/torch rendezvous env the operator injected
GET /exit?exitCode=N   respond, then exit the process with code N

Listens on $PORT (local kubelet) or --port (default 2222, the TFJob port).
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import threading
import time

from flask import Flask, request

APP = Flask(__name__)


def runconfig_from_tf_config(tf_config: str) -> dict:
    cfg = json.loads(tf_config) if tf_config else {}
    cluster = cfg.get("cluster", {}) or {}
    task = cfg.get("task", {}) or {}
    ttype = task.get("type", "")
    tid = int(task.get("index", 0) or 0)
    if ttype == "evaluator":
        return {"task_type": "evaluator", "task_id": 0, "cluster_spec": {}, "is_chief": False, "master": "",
                "num_worker_replicas": 0, "num_ps_replicas": 0}
    if "chief" in cluster or "master" in cluster:
        is_chief = ttype in ("chief", "master")
    else:
        is_chief = ttype == "worker" and tid == 0
    addr = (cluster.get(ttype) or [""])[tid] if ttype in cluster else ""
    return {"task_type": ttype, "task_id": tid, "cluster_spec": cluster, "is_chief": is_chief,
            "master": f"grpc://{addr}" if addr else "",
            "num_worker_replicas": len(cluster.get("worker", [])) + len(cluster.get("chief", []))
            + len(cluster.get("master", [])),
            "num_ps_replicas": len(cluster.get("ps", []))}


@APP.route("/")
def index():
    return "hello world"


@APP.route("/tfconfig", methods=["GET"])
def tf_config():
    return os.environ.get("TF_CONFIG", "")


@APP.route("/runconfig", methods=["GET"])
def run_config():
    return json.dumps(runconfig_from_tf_config(os.environ.get("TF_CONFIG", "")))


@APP.route("/env", methods=["GET"])
def env():
    keys = ("MASTER_ADDR", "MASTER_PORT", "WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "TOA_ROLE",
            "TOA_PS_HOSTS", "HIP_VISIBLE_DEVICES", "TOA_REPLICA_TYPE", "TOA_REPLICA_INDEX")
    out = {k: os.environ[k] for k in keys if k in os.environ}
    out.update({k: v for k, v in os.environ.items() if k.startswith(("NCCL_", "RCCL_"))})
    return json.dumps(out)


@APP.route("/exit", methods=["GET"])
def exit_handler():
    code = int(request.args.get("exitCode", 0))

    def _die():
        time.sleep(0.2)
        os._exit(code)

    threading.Thread(target=_die, daemon=True).start()
    return f"Shutting down with exitCode {code}"


def main(argv=None):
    logging.basicConfig(level=logging.INFO)
    p = argparse.ArgumentParser(description="TFJob test server.")
    p.add_argument("--port", type=int, default=int(os.environ.get("PORT", 2222)))
    a = p.parse_args(argv)
    logging.getLogger("werkzeug").setLevel(logging.WARNING)
    APP.run(debug=False, host="127.0.0.1" if "PORT" in os.environ else "0.0.0.0", port=a.port)


if __name__ == "__main__":
    main()

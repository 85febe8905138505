"""Starts the rank processes of the multi-process GPU tests (tests/test_gpu_multiproc.py).

conftest.py starts this helper when the session begins, before any test touches the GPU: a
process that has initialised the GPU must not fork + exec another program, so the pytest
process never starts the ranks itself.  This helper never loads HIP.

Protocol (one JSON object per line): the request {"cmds": [argv, ...], "timeout": seconds,
"env": {...}} starts one process per argv (its own session, output to a temporary file); the
reply {"rc": [...], "out": [...]} carries each exit status and the tail of its output.  A rank
that fails makes its peers fail within seconds (the shm transport notices the exited pid); past
the timeout, or `grace` (default 20) seconds after the first failure, the remaining ranks' process
groups are killed.
EOF on stdin ends the helper.
"""
import json
import os
import signal
import subprocess
import sys
import tempfile
import time


def run(req):
    env = dict(os.environ)
    env.update(req.get("env", {}))
    # every rank shares the one GPU: past 6 processes with HIP's default queues its scheduler
    # time-slices whole processes (bench.py's shared_gpu_queues)
    cap = 4 if len(req["cmds"]) <= 6 else 1
    env["GPU_MAX_HW_QUEUES"] = str(min(int(env.get("GPU_MAX_HW_QUEUES") or 4), cap))
    procs, logs = [], []
    for argv in req["cmds"]:
        f = tempfile.TemporaryFile()
        procs.append(subprocess.Popen(argv, stdout=f, stderr=subprocess.STDOUT, env=env,
                                      start_new_session=True))
        logs.append(f)
    deadline = time.time() + float(req.get("timeout", 240))
    grace = float(req.get("grace", 20))
    first_fail = None
    rcs = [None] * len(procs)
    while any(rc is None for rc in rcs):
        rcs = [p.poll() for p in procs]
        now = time.time()
        if first_fail is None and any(rc not in (None, 0) for rc in rcs):
            first_fail = now
        if now > deadline or (first_fail is not None and now - first_fail > grace):
            for p, rc in zip(procs, rcs):
                if rc is None:
                    try:
                        os.killpg(p.pid, signal.SIGKILL)
                    except OSError:
                        pass
            for p in procs:
                p.wait()
            rcs = [p.returncode for p in procs]
            break
        time.sleep(0.05)
    outs = []
    for f in logs:
        f.seek(0)
        outs.append(f.read().decode(errors="replace")[-6000:])
        f.close()
    return {"rc": rcs, "out": outs}


def main():
    for line in sys.stdin:
        line = line.strip()
        if not line:
            continue
        try:
            reply = run(json.loads(line))
        except Exception as e:  # noqa: BLE001 - reported to the test
            reply = {"rc": [-1], "out": [f"launcher: {type(e).__name__}: {e}"]}
        sys.stdout.write(json.dumps(reply) + "\n")
        sys.stdout.flush()


if __name__ == "__main__":
    main()

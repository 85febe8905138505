"""CPU: the rank launcher of the multi-process GPU tests (tests/rank_launcher.py) — exit codes and
output come back per rank, and a failing rank ends its peers instead of leaving them waiting."""
import os
import sys
import time

from conftest import RankLauncher

HERE = os.path.dirname(os.path.abspath(__file__))


def _launcher():
    import subprocess
    return subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "rank_launcher.py")],
                            stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)


def test_launcher_runs_ranks_and_reports():
    p = _launcher()
    try:
        rl = RankLauncher(p)
        cmds = [[sys.executable, "-c", f"print('rank {r}'); raise SystemExit({r})"] for r in range(3)]
        rcs, outs = rl.run(cmds, timeout=60)
        assert rcs == [0, 1, 2]
        assert [o.strip() for o in outs] == ["rank 0", "rank 1", "rank 2"]
    finally:
        p.stdin.close()
        p.wait(timeout=30)


def test_launcher_ends_peers_of_a_failed_rank():
    p = _launcher()
    try:
        rl = RankLauncher(p)
        cmds = [[sys.executable, "-c", "raise SystemExit(3)"],
                [sys.executable, "-c", "import time; time.sleep(120)"]]
        t0 = time.time()
        p.stdin.write('{"cmds": %s, "timeout": 60, "grace": 1}\n' % str(cmds).replace("'", '"'))
        p.stdin.flush()
        import json
        reply = json.loads(p.stdout.readline())
        assert reply["rc"][0] == 3 and reply["rc"][1] != 0
        assert time.time() - t0 < 30
    finally:
        p.stdin.close()
        p.wait(timeout=30)

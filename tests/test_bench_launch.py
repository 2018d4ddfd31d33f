"""bench.py --gpus N without a launcher starts the N-rank run itself
(torch.distributed.run as a child process, before anything touches the GPU),
relays rank 0's JSON line and returns the child's exit code.  CPU only."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class FakeProc:
    def __init__(self, rc, out):
        self.returncode, self.stdout = rc, out


def test_relaunch_command_and_relay(capsys):
    sys.path.insert(0, REPO)
    import bench
    seen = {}

    def run(cmd, env=None, stdout=None, text=None):
        seen["cmd"], seen["env"] = cmd, env
        return FakeProc(3, 'noise\n{"metric": "m", "n_gpus": 4}\n')

    argv = ["--gpus", "4", "--steps", "3", "--workload", "c3"]
    rc = bench.maybe_relaunch(argv, 4, env={"PATH": "/bin"}, run=run)
    assert rc == 3
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-len(argv):] == argv and cmd[-len(argv) - 1].endswith("bench.py")
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    out = capsys.readouterr().out.strip().splitlines()
    assert out == ['{"metric": "m", "n_gpus": 4}'] and json.loads(out[0])["n_gpus"] == 4


def test_no_relaunch_for_one_gpu_or_under_a_launcher():
    sys.path.insert(0, REPO)
    import bench
    assert bench.maybe_relaunch(["--gpus", "1"], 1, env={}) is None
    assert bench.maybe_relaunch(["--gpus", "8"], 8, env={"WORLD_SIZE": "8"}) is None


def test_parent_never_imports_torch():
    """The relaunching parent must not initialise the GPU (an exec-like hand-off
    after GPU init is forbidden on the pool): bench's import and the relaunch
    decision load no torch at all."""
    code = ("import sys; sys.path.insert(0, %r); import bench\n"
            "class P: returncode = 0; stdout = ''\n"
            "rc = bench.maybe_relaunch(['--gpus', '2'], 2, env={}, run=lambda *a, **k: P())\n"
            "assert rc == 0 and 'torch' not in sys.modules, sorted(m for m in sys.modules if 'torch' in m)\n" % REPO)
    subprocess.run([sys.executable, "-c", code], check=True)

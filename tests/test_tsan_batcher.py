"""CPU: ThreadSanitizer build of the host micro-batcher (weaviate_amd/csrc/
batcher.hip, the coalescing of concurrent SearchByVector callers --
shard_read.go:415-424) driven by 48 threads against a CPU mock of the batch
search while another thread retunes batch_window_us / batch_max
(tools/tsan_batcher.sh).  A data race aborts the run; every result must equal
a serial search of the same query."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not (os.path.exists("/opt/rocm/lib/llvm/bin/clang++") or shutil.which("clang++")),
                    reason="needs clang++ with TSan")
def test_batcher_tsan(tmp_path):
    env = dict(os.environ, TMPDIR=str(tmp_path))
    r = subprocess.run(["bash", os.path.join(REPO, "tools", "tsan_batcher.sh"), "48", "60"], capture_output=True,
                       text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
    assert "0 mismatches" in r.stdout and "48 threads x 60 calls" in r.stdout

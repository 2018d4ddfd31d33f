"""CPU: ASan + UBSan build of the LSM segment reader (host code of
weaviate_amd/csrc/lsm_segment.hip) fuzzed with mutated segment files --
tools/asan_lsm.sh (truncation, bit flips, huge length fields, moved index
start, bad checksums).  Any out-of-bounds access aborts the run."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++ with ASan")
def test_lsm_reader_asan_fuzz(tmp_path):
    env = dict(os.environ, TMPDIR=str(tmp_path))
    r = subprocess.run(["bash", os.path.join(REPO, "tools", "asan_lsm.sh"), "3000"], capture_output=True, text=True,
                       env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "lsm_fuzz: 3000 iterations" in r.stdout
    ok = int(r.stdout.split("iterations, ")[1].split(" parses ok")[0])
    assert ok > 0  # some mutants still parse: the restore path (collect + gather) ran

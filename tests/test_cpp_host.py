"""The C++ host mirror (gelly-streaming_amd/host/gelly/*.hpp) replaying the reference's own tests
(DisjointSetTest, ConnectedComponentsTest, the example's default data) through the C ABI on the GPU."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "build", "test_host_mirror")


def test_cpp_mirror_builds():
    """CPU: the headers compile against include/gelly_cc.h and link against the in-tree library."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")], check=True)
    assert os.path.exists(BIN)


@pytest.mark.gpu
def test_cpp_mirror_reference_tests():
    # rebuilt here (-B): a binary that arrived with the snapshot may not be executable on the GPU box
    subprocess.run(["make", "-s", "-B", "-C", os.path.join(ROOT, "tests", "cpp"), "build/test_host_mirror"], check=True)
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("PASS ") >= 10

"""Race / memory-error detection for the native host runtime (the reference has
no race detection; TF1's Hogwild PS updates are racy by design). The parameter server, token
queue, conditional accumulators, checkpoint IO and batch prefetcher are compiled together with
a multi-threaded stress driver under ThreadSanitizer and AddressSanitizer+UBSan
(tools/sanitize_runtime.sh) and must run clean with exact protocol results."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++ with libtsan/libasan")
def test_runtime_stress_under_tsan_and_asan(tmp_path):
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize_runtime.sh"), str(tmp_path)],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    for log in ("tsan.log", "asan.log"):
        text = (tmp_path / log).read_text()
        assert "PASS" in text and "WARNING: ThreadSanitizer" not in text and "ERROR: AddressSanitizer" not in text
        assert "runtime error" not in text  # UBSan

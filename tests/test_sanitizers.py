"""Sanitizer builds of the host code (the reference carries ASan
flags in CMakeLists.txt:37-39): libnxec's host side compiled with
AddressSanitizer (+LeakSanitizer), UndefinedBehaviorSanitizer and
ThreadSanitizer, driven by tests/cpp/host_sanity_test.cc on the CPU --
GF(2^8) planning over many (n,k), argument validation of the entry points,
the CodingOptions defaults source raced by 8 threads, Chunk / arena ownership
and the host worker pool under 8 concurrent RSCode callers.  No GPU: every
compute call must fail cleanly (NXEC_ERR_NODEV)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

ENV = {
    "asan": {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1",
             "LSAN_OPTIONS": f"suppressions={ROOT}/tests/cpp/lsan.supp"},
    "ubsan": {"UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"},
    "tsan": {"TSAN_OPTIONS": "ignore_noninstrumented_modules=1:halt_on_error=1"},
}


@pytest.mark.parametrize("kind", ["asan", "ubsan", "tsan"])
def test_host_code_under_sanitizer(kind):
    binary = os.path.join(ROOT, "build", "san", kind, "host_sanity_test")
    _run(kind, binary)


@pytest.mark.parametrize("kind", ["asan", "ubsan"])
def test_reference_chunk_sequences_under_sanitizer(kind):
    """The reference's shallow Chunk copies (chunk_manager.cc:176-178, :1275,
    :1498, proxy_file_ops.cc:585, agent.cc:366, container_manager.cc:252)
    replayed against csrc/coding/chunk.hh: aliases point at the original
    buffers, LeakSanitizer reports no leak and ASan no double free."""
    _run(kind, os.path.join(ROOT, "build", "san", kind, "chunk_replay_test"))


def _run(kind, binary):
    if not os.path.exists(binary):  # built by __graft_entry__.build(); build here when missing
        jobs = str(min(os.cpu_count() or 8, 16))
        r = subprocess.run(["make", "-C", ROOT, f"-j{jobs}", kind], capture_output=True, text=True, timeout=900)
        assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, **ENV[kind], HIP_VISIBLE_DEVICES="")
    r = subprocess.run([binary], capture_output=True, text=True, timeout=300, env=env)
    report = r.stdout[-3000:] + r.stderr[-6000:]
    assert r.returncode == 0, report
    assert "PASSED 0 failures" in r.stdout, report
    for marker in ("ERROR: AddressSanitizer", "ERROR: LeakSanitizer", "runtime error:", "WARNING: ThreadSanitizer"):
        assert marker not in r.stderr, report

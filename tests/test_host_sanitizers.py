"""Race / memory-error detection for the native host runtime ("race detection /
sanitizers"): the multi-threaded CSV reader and as-of join are compiled with AddressSanitizer +
UBSan and, separately, ThreadSanitizer, and a C++ harness (tools/sanitize/host_runtime_check.cpp)
drives them through edge cases and thread counts on the CPU.  GPU-side sanitizers are not
available on this pool; device code is covered by the fp64 oracle tests instead."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "tools", "sanitize", "host_runtime_check.cpp"),
       os.path.join(ROOT, "llm_driven_multi_factor_model_amd", "csrc_host", "csv_panel.cpp"),
       os.path.join(ROOT, "llm_driven_multi_factor_model_amd", "csrc_host", "asof.cpp"),
       os.path.join(ROOT, "llm_driven_multi_factor_model_amd", "csrc_host", "csv_write.cpp")]


def _build_and_run(tmp_path, flags, env_extra):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path / "host_check")
    p = subprocess.run([cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread",
                        *flags, *SRC, "-o", exe], capture_output=True, text=True)
    if p.returncode != 0 and "sanitize" in p.stderr:
        pytest.skip(f"sanitizer runtime unavailable: {p.stderr[-300:]}")
    assert p.returncode == 0, p.stderr[-3000:]
    env = dict(os.environ, **env_extra)
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "ok" in r.stdout


def test_host_runtime_asan_ubsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"],
                   {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1",
                    "UBSAN_OPTIONS": "print_stacktrace=1:halt_on_error=1"})


def test_host_runtime_tsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=thread"], {"TSAN_OPTIONS": "halt_on_error=1"})

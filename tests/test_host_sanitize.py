"""The host planning code of libmirsha (alias detection, size-class order,
block partition, direct-mode lane planner) under AddressSanitizer and
UndefinedBehaviorSanitizer, on CPU: tests/cpp/host_planning_asan.cpp includes
mirbft_amd/csrc/mirsha.cpp, stubs the kernel launchers, and checks every result
against a plain reference over random and edge-case inputs. (GPU sanitizers are
not available on this pool; host code is where they apply.)"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CPP = os.path.join(HERE, "cpp")


def test_host_planning_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", CPP, "asan"], check=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(CPP, "build", "host_planning_asan")], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "all checks passed" in r.stdout


def test_host_planning_under_tsan():
    """The same harness under ThreadSanitizer: the planning phases run on the
    worker pool at these sizes (>= 2^18 items), so a race between its threads is
    reported (the reference's CI runs ginkgo --race)."""
    subprocess.run(["make", "-s", "-C", CPP, "tsan"], check=True, timeout=600)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([os.path.join(CPP, "build", "host_planning_tsan")], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "all checks passed" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr

"""The C++ host mirror (include/mirbft/processor.hpp) builds (CPU) and passes
its reference-shaped specs against the GPU engine (GPU)."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CPP = os.path.join(HERE, "cpp")


def _build():
    subprocess.run(["make", "-s", "-C", CPP], check=True)
    return os.path.join(CPP, "build", "test_processor")


def test_cpp_mirror_builds():
    assert os.path.exists(_build())


@pytest.mark.gpu
def test_cpp_mirror_specs_on_gpu():
    out = subprocess.run([_build()], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr + out.stdout
    assert "all specs passed" in out.stdout

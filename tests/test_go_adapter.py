"""The committed Go drop-in (go/) stays consistent with the C ABI and the
reference tree, on CPU (no Go toolchain in this image, so it is checked
textually): every libmirsha symbol and constant the cgo file uses is declared
in include/mirsha.h, and go/wiring.patch applies cleanly to the reference."""
import os
import re
import shutil
import subprocess

import pytest

from mirbft_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO = os.path.join(ROOT, "go", "pkg", "processor", "gpuhash.go")
REF = "/root/reference"


def test_cgo_uses_only_declared_abi():
    src = open(GO).read()
    header = open(L.HEADER_PATH).read()
    used = set(re.findall(r"\bC\.(msha_\w+|MSHA_\w+)", src))
    assert {"msha_ctx_create_err", "msha_digest_batch", "msha_pinned_alloc", "msha_last_error"} <= used
    for name in used:
        assert re.search(r"\b%s\b" % name, header), f"{name} not in include/mirsha.h"
    for fn in set(re.findall(r"\bC\.(msha_\w+)\(", src)):
        assert fn in L.SIGNATURES, fn


def test_cgo_signatures_match_header_arity():
    """Each C.msha_* call in the Go file passes as many arguments as the header declares."""
    src = open(GO).read()
    header = open(L.HEADER_PATH).read()
    for m in re.finditer(r"C\.(msha_\w+)\(", src):
        name = m.group(1)
        depth, i, args = 1, m.end(), 1
        while depth:
            c = src[i]
            depth += c == "("
            depth -= c == ")"
            args += c == "," and depth == 1
            i += 1
        if src[m.end():i - 1].strip() == "":
            args = 0
        decl = re.search(r"^[\w \*]*\b%s\s*\(([^)]*)\);" % name, header, re.M).group(1)
        nparams = 0 if decl.strip() in ("", "void") else decl.count(",") + 1
        assert args == nparams, (name, args, nparams)


@pytest.mark.skipif(not os.path.isdir(REF) or not shutil.which("patch"), reason="reference tree absent")
def test_wiring_patch_applies_to_reference(tmp_path):
    for rel in ("mirbft.go", "pkg/processor/clients.go", "pkg/testengine/recorder.go"):
        dst = tmp_path / rel
        dst.parent.mkdir(parents=True, exist_ok=True)
        shutil.copy(os.path.join(REF, rel), dst)
    r = subprocess.run(["patch", "-p1", "-i", os.path.join(ROOT, "go", "wiring.patch")], cwd=tmp_path,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    clients = (tmp_path / "pkg/processor/clients.go").read_text()
    assert "func (c *Client) proposeDigest(reqNo uint64, data, digest []byte)" in clients
    assert "ProcessHashActionsGPU(n.processorConfig.GPUHasher, actions)" in (tmp_path / "mirbft.go").read_text()
    assert "MIRBFT_TEST_GPU_HASH" in (tmp_path / "pkg/testengine/recorder.go").read_text()

"""The committed Go drop-in (go/) stays consistent with the C ABI and the
reference tree, on CPU (no Go toolchain in this image, so it is checked
textually): every libmirsha symbol and constant the cgo file uses is declared
in include/mirsha.h, go/wiring.patch applies cleanly to the reference, and the
cgo file (build tag mirsha) and its no-cgo stub (no tag) declare the same
exported API, so the patched tree builds with and without libmirsha."""
import os
import re
import shutil
import subprocess

import pytest

from mirbft_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GODIR = os.path.join(ROOT, "go", "pkg", "processor")
GO = os.path.join(GODIR, "gpuhash.go")
STUB = os.path.join(GODIR, "gpuhash_stub.go")
API = os.path.join(GODIR, "gpuhash_api.go")
REF = "/root/reference"


def test_cgo_uses_only_declared_abi():
    src = open(GO).read()
    header = open(L.HEADER_PATH).read()
    used = set(re.findall(r"\bC\.(msha_\w+|MSHA_\w+)", src))
    assert {"msha_ctx_create_err", "msha_digest_batch", "msha_pinned_alloc", "msha_last_error_copy"} <= used
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


def _build_tag(path):
    """The file's build constraint: (go:build expr, +build expr) before the package clause."""
    head = open(path).read().split("\npackage ", 1)[0]
    gb = re.search(r"^//go:build (.+)$", head, re.M)
    pb = re.search(r"^// \+build (.+)$", head, re.M)
    return (gb.group(1).strip() if gb else None, pb.group(1).strip() if pb else None)


def _exported(path):
    """Exported top-level declarations of a Go file: funcs/methods with their
    signatures (receiver reduced to its type, parameter names kept), and types."""
    src = open(path).read()
    decls = set()
    for m in re.finditer(r"^func (?:\((\w+) ([^)]*)\) )?([A-Z]\w*)(\(.*?) ?\{\}?$", src, re.M):
        recv, name, sig = m.group(2), m.group(3), " ".join(m.group(4).split())
        decls.add(("func", recv or "", name, sig))
    for m in re.finditer(r"^type ([A-Z]\w*) ", src, re.M):
        decls.add(("type", "", m.group(1), ""))
    for m in re.finditer(r"^(?:var|const) ([A-Z]\w*)", src, re.M):
        decls.add(("var", "", m.group(1), ""))
    return decls


def _toplevel_names(path):
    src = open(path).read()
    names = set(re.findall(r"^func (?:\(\w+ \*?(\w+)\) )?(\w+)\(", src, re.M))
    names |= {("", n) for n in re.findall(r"^(?:type|var|const) (\w+)", src, re.M)}
    return names


def test_go_files_build_tagged():
    """gpuhash.go links libmirsha (cgo), so only `-tags mirsha` builds compile it;
    the stub takes its place otherwise, and the shared file carries no tag and no cgo."""
    assert _build_tag(GO) == ("mirsha", "mirsha")
    assert _build_tag(os.path.join(GODIR, "gpuhash_test.go")) == ("mirsha", "mirsha")
    assert _build_tag(STUB) == ("!mirsha", "!mirsha")
    assert _build_tag(os.path.join(GODIR, "gpuhash_stub_test.go")) == ("!mirsha", "!mirsha")
    assert _build_tag(API) == (None, None)
    for path in (STUB, API, os.path.join(GODIR, "gpuhash_stub_test.go")):
        assert 'import "C"' not in open(path).read(), path
    # Go 1.15 reads only the +build line; it must come before the package clause
    # and be followed by a blank line.
    for path in (GO, STUB):
        src = open(path).read()
        assert re.search(r"^// \+build [!\w]+\n\n", src, re.M), path


def test_go_stub_declares_the_same_api():
    real, stub = _exported(GO), _exported(STUB)
    assert real == stub, (real ^ stub)
    names = {d[2] for d in real}
    assert {"GPUHasher", "NewGPUHasher", "Close", "RequestDigests", "ProcessHashActionsGPU"} <= names
    # Nothing is declared twice in either build (the shared file + one of the two).
    api = _toplevel_names(API)
    assert not (api & _toplevel_names(GO)), api & _toplevel_names(GO)
    assert not (api & _toplevel_names(STUB)), api & _toplevel_names(STUB)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree absent")
def test_patched_tree_uses_only_declared_processor_api():
    """Every processor.X the wiring patch adds is declared by the reference's
    pkg/processor or by BOTH builds of the drop-in, so the patched tree compiles
    with and without the mirsha tag."""
    patch = open(os.path.join(ROOT, "go", "wiring.patch")).read()
    added = "\n".join(l[1:] for l in patch.splitlines() if l.startswith("+") and not l.startswith("+++"))
    used = set(re.findall(r"\bprocessor\.([A-Z]\w*)", added))
    assert {"GPUHasher", "ProcessHashActionsGPU", "NewGPUHasher", "ProposedRequest"} <= used
    ref_pkg = set()
    pdir = os.path.join(REF, "pkg", "processor")
    for f in os.listdir(pdir):
        if f.endswith(".go") and not f.endswith("_test.go"):
            ref_pkg |= {n for _, n in _toplevel_names(os.path.join(pdir, f))}
    api = {n for _, n in _toplevel_names(API)}
    for build in (GO, STUB):
        have = ref_pkg | api | {n for _, n in _toplevel_names(build)}
        missing = used - have
        assert not missing, (build, missing)
    # Methods the patch calls on processor values: Client.ProposeBatch (shared file)
    # and Client.proposeDigest (added to clients.go by the patch itself).
    assert ("Client", "ProposeBatch") in _toplevel_names(API)
    assert "func (c *Client) proposeDigest(" in added

"""Experiment builds never pose as the product:
no tools/ script writes over mirbft_amd/libmirsha.so -- variants are built outside
the package (tools/ab_build.sh) and loaded through MSHA_LIB_PATH -- and a library
loaded that way is reported as foreign, so GPU test sessions and bench.py refuse
it unless MSHA_ALLOW_FOREIGN_LIB=1. CPU only (msha_build_id needs no GPU)."""
import glob
import os
import re
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_no_script_writes_the_product_library():
    bad = []
    for f in sorted(glob.glob(os.path.join(ROOT, "tools", "*.sh")) + glob.glob(os.path.join(ROOT, "tools", "*.py"))):
        for i, line in enumerate(open(f, errors="replace"), 1):
            code = line.split("#", 1)[0] if f.endswith(".sh") else line
            # cp / mv / install / ln / redirection with the product path as destination
            if re.search(r"\b(cp|mv|install|ln)\b[^;&|]*\s\S*mirbft_amd/libmirsha\.so\s*($|[;&|])", code) or \
                    re.search(r">\s*\S*mirbft_amd/libmirsha\.so", code):
                bad.append("%s:%d: %s" % (os.path.relpath(f, ROOT), i, line.strip()))
    assert not bad, "scripts that overwrite the product library:\n" + "\n".join(bad)


def test_variant_dir_stays_off_the_gpu_box():
    ignore = open(os.path.join(ROOT, ".gpurunignore")).read().split()
    assert "./build_ab" in ignore
    assert not os.path.exists(os.path.join(ROOT, "build_ab")) or not glob.glob(os.path.join(ROOT, "build_ab", "*.so"))


def _probe(env_extra):
    code = ("import json, sys; sys.path.insert(0, %r)\n"
            "from mirbft_amd import _lib\n"
            "b = _lib.build_id()\n"
            "try:\n    _lib.require_tree_build('probe'); refused = False\n"
            "except RuntimeError:\n    refused = True\n"
            "print(json.dumps({'matches_tree': b['matches_tree'], 'path': b['path'], 'refused': refused}))" % ROOT)
    env = dict(os.environ)
    env.pop("MSHA_LIB_PATH", None)
    env.pop("MSHA_ALLOW_FOREIGN_LIB", None)
    env.update(env_extra)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    import json
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_lib_path_variant_is_foreign(tmp_path):
    prod = os.path.join(ROOT, "mirbft_amd", "libmirsha.so")
    own = _probe({})
    assert own["matches_tree"] and not own["refused"], own
    v = tmp_path / "variant.so"
    shutil.copy(prod, v)  # even a byte-identical copy is not the tree's library path
    got = _probe({"MSHA_LIB_PATH": str(v)})
    assert got["path"] == str(v) and not got["matches_tree"] and got["refused"], got
    allowed = _probe({"MSHA_LIB_PATH": str(v), "MSHA_ALLOW_FOREIGN_LIB": "1"})
    assert not allowed["refused"]

import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


def pytest_report_header(config):
    """Name the library build the session runs (msha_build_id), so a failure log says
    which build produced it."""
    try:
        from mirbft_amd import _lib
        b = _lib.build_id()
        return "libmirsha: %s (tree src %s, %s)" % (b["id"], b["tree_src"],
                                                    "the tree's build" if b["matches_tree"] else "NOT the tree's build")
    except Exception as ex:  # noqa: BLE001 -- a header must not fail the session
        return "libmirsha: not loadable here (%s)" % ex


@pytest.hookimpl(trylast=True)
def pytest_collection_modifyitems(config, items):
    """A session that selected any GPU test, on a library that is not the tree's own
    build (an experiment's .so, or MSHA_LIB_PATH naming a variant), is refused: its
    results would be reported as the product's. trylast: runs after -m / -k
    deselection, so `items` is what will run. MSHA_ALLOW_FOREIGN_LIB=1 runs it anyway
    (A/B runs of a variant build)."""
    if not any(it.get_closest_marker("gpu") for it in items) or os.environ.get("MSHA_ALLOW_FOREIGN_LIB") == "1":
        return
    try:
        from mirbft_amd import _lib
        b = _lib.build_id()
    except Exception as ex:  # noqa: BLE001 -- a missing / pre-ABI-9 library: say so, not an INTERNALERROR
        raise pytest.UsageError("GPU tests selected but libmirsha's build id is unreadable (%s): build it with "
                                "make -C mirbft_amd/csrc" % ex)
    if not b["matches_tree"]:
        raise pytest.UsageError("%s is not this tree's build (%s; tree src %s): rebuild it "
                                "(make -C mirbft_amd/csrc) or set MSHA_ALLOW_FOREIGN_LIB=1"
                                % (b["path"], b["id"], b["tree_src"]))


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def kat():
    return load_golden("kat.json")


@pytest.fixture(scope="session")
def lengths_golden():
    from mirbft_amd.workloads import SEED, random_bytes
    g = load_golden("lengths.json")
    out = []
    for e in g["messages"]:
        if "msg_hex" in e:
            m = bytes.fromhex(e["msg_hex"])
        else:
            m = random_bytes(SEED ^ 0x60, e["len"] << 20, e["len"]).tobytes()
        assert len(m) == e["len"]
        out.append((m, bytes.fromhex(e["sha256"])))
    return out


@pytest.fixture(scope="session")
def actions_golden():
    g = load_golden("actions.json")
    return [(a["name"], a["kind"], [bytes.fromhex(p) for p in a["parts_hex"]], bytes.fromhex(a["sha256"]))
            for a in g["actions"]]


@pytest.fixture(scope="session")
def engine():
    import torch  # one HIP runtime per process: torch's, loaded before libmirsha (see mirbft_amd/_lib.py)
    torch.cuda.init()
    from mirbft_amd import Engine
    e = Engine(1)
    yield e
    e.close()

"""the testengine's checkpoint value chain (NodeState.Snap /
Apply, recorder.go:288-353) computed on the GPU, node-parallel per interval,
bit-exact against a streaming hashlib restatement of NodeState."""
import hashlib
import random

import pytest

from mirbft_amd import GPUHasher, checkpoint_hashes

pytestmark = pytest.mark.gpu


def test_checkpoint_chain_4_nodes(engine):
    hasher = GPUHasher(engine)
    rnd = random.Random(11)
    nodes = 4
    streams = [hashlib.sha256() for _ in range(nodes)]   # Hasher.New() (recorder.go:420)
    prev = [None] * nodes
    for interval in range(20):
        committed = [[hashlib.sha256(b"%d-%d-%d" % (n, interval, j)).digest()
                      for j in range(rnd.randrange(0, 41))] for n in range(nodes)]
        got = checkpoint_hashes(hasher, [(prev[n], committed[n]) for n in range(nodes)])
        for n in range(nodes):
            for d in committed[n]:
                streams[n].update(d)                      # Apply (:348)
            exp = streams[n].digest()                     # Snap: Sum(nil) (:298)
            assert got[n] == exp, (n, interval)
            streams[n] = hashlib.sha256(exp)              # New + Write(CheckpointHash) (:299-300)
            prev[n] = exp


def test_checkpoint_many_intervals_one_call(engine):
    hasher = GPUHasher(engine)
    rnd = random.Random(12)
    intervals = []
    for i in range(5000):
        prev = None if i % 7 == 0 else hashlib.sha256(b"p%d" % i).digest()
        intervals.append((prev, [hashlib.sha256(b"%d/%d" % (i, j)).digest() for j in range(rnd.randrange(0, 60))]))
    got = checkpoint_hashes(hasher, intervals)
    for (prev, ds), g in zip(intervals, got):
        assert g == hashlib.sha256((prev or b"") + b"".join(ds)).digest()
    assert checkpoint_hashes(hasher, []) == []

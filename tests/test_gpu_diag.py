"""GPU checks of the diagnostics and of the Python wrapper's argument checks:
msha_clock_probe (bench.py's effective_clock_ghz) and the device entry points'
tensor validation (a wrong dtype, device layout or a short output raises
before any pointer reaches the GPU)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_clock_probe_reads_a_plausible_clock(engine):
    c = engine.clock_probe(48)
    assert 0.5 < c["ghz_min"] <= c["ghz_median"] <= c["ghz_max"] < 3.5, c
    assert c["workgroups"] >= 256 * 8 and c["blocks_per_lane"] == 48
    assert c["kernel_ms"] > 0 and 1 < c["gblocks_per_s"] < 60, c
    from mirbft_amd import MshaError
    with pytest.raises(MshaError):
        engine.clock_probe(0)


def test_device_arguments_validated(engine):
    import torch
    dev = torch.device("cuda:0")
    arena = torch.zeros(4096, dtype=torch.uint8, device=dev)
    off = torch.zeros(4, dtype=torch.int64, device=dev)
    ln = torch.full((4,), 10, dtype=torch.int64, device=dev)
    out = torch.zeros((4, 32), dtype=torch.uint8, device=dev)
    with pytest.raises(ValueError, match="8-byte"):
        engine.digest_batch_device(arena, off.int(), ln, out)
    with pytest.raises(ValueError, match="needs 128"):
        engine.digest_batch_device(arena, off, ln, out[:3])
    with pytest.raises(ValueError, match="contiguous"):
        engine.digest_batch_device_planned(arena, torch.zeros(8, dtype=torch.int64, device=dev)[::2], ln, out)
    with pytest.raises(ValueError, match="entries"):
        engine.digest_batch_device(arena, off, ln[:3], out)
    with pytest.raises(ValueError, match="4-byte"):
        engine.digest_batch_device(arena, off, ln, out, order=torch.zeros(4, dtype=torch.int64, device=dev))
    with pytest.raises(ValueError, match="cuda:0"):
        engine.digest_of_digests_device(out.cpu(), torch.zeros(1, dtype=torch.int32, device=dev),
                                        torch.zeros(2, dtype=torch.int64, device=dev), out)
    # and the valid call still runs
    engine.digest_batch_device(arena, off * 16, ln, out)
    engine.device_status()
    import hashlib
    assert bytes(out[0].cpu().numpy()) == hashlib.sha256(bytes(10)).digest()

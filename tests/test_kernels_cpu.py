"""Resource checks of the built device code (CPU only: the kernel descriptors of
libspai.so's gfx950 code object, scripts/kernel_regs.py).  The hot kernels must use
no scratch memory: a register array indexed by a loop that stayed rolled lands on
the scratch stack and silently costs the forward several times its time (round 6:
one build of the C4 forward spilled its B/A rings there at S = 4).  The C4 forward's
register footprint must also leave a tree-kernel wave room beside it on the SIMD
(<= 464 of 512), which is what lets one search chain's select run
under the other chain's forward."""
import os
import sys

import pytest

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, "scripts"))
LIB = os.path.join(REPO, "self-play-ai_amd", "libspai.so")

HOT = ["k_forwardILb0E", "k_forwardILb1E", "k_selectILb0E", "k_expand_selectILb0E", "k_advance", "k_chess_forward",
       "k_cleaf", "k_cexpand", "k_legal4", "k_apply4", "k_encodeILb1E"]


@pytest.fixture(scope="module")
def descriptors():
    if not os.path.exists(LIB):
        pytest.skip("libspai.so not built")
    import kernel_regs
    return kernel_regs.kernels(LIB)


@pytest.mark.parametrize("kernel", HOT)
def test_hot_kernels_use_no_scratch(descriptors, kernel):
    hits = {n: f for n, f in descriptors.items() if kernel in n}
    assert hits, kernel
    for n, f in hits.items():
        assert int(f["private_segment_fixed_size"]) == 0, (n, f["private_segment_fixed_size"])


def test_c4_forward_register_budget(descriptors):
    for n, f in descriptors.items():
        if "k_forwardILb0E" in n:
            assert int(f["vgpr_count"]) <= 464, (n, f["vgpr_count"])
            assert int(f["vgpr_spill_count"]) == 0, (n, f["vgpr_spill_count"])

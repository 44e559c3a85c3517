"""The built gfx950 code object has no store-data overwrite hazard
(stochquant_amd/isa_check.py): no 12/16-byte VMEM store is
followed within two wait states by a VALU write of its data registers.  Round
2's one-accumulator frame variant had five such stores (buffer stores with an
SGPR soffset, which the compiler does not pad) and stored wrong first
components in a few lanes; CPU only, it reads the ELF."""
import os
import shutil

import pytest

from conftest import ROOT


def test_no_store_data_overwrite_hazard(sqlib):
    from stochquant_amd import isa_check
    if not shutil.which(os.path.join(isa_check.LLVM, "llvm-objdump")):
        pytest.fail("llvm-objdump missing from the ROCm image")
    text = isa_check.disassemble(os.path.join(ROOT, "stochquant_amd", "lib", "libstochquant.so"))
    assert text.count("buffer_store_dwordx4") > 100      # the kernels are there
    bad = isa_check.store_data_hazards(text)
    assert bad == [], bad[:5]


def test_checker_sees_the_round2_pattern():
    """The checker flags the exact sequence the failing variant had."""
    from stochquant_amd import isa_check
    text = """0000000000001000 <k>:
	buffer_store_dwordx4 v[2:5], v54, s[40:43], s54 offen sc0 sc1 // 000000372D6C: E07CD000 360A0236
	v_max3_f32 v2, v27, v28, v29 // 000000372D74: D1D30002 0476391B
	buffer_store_dwordx4 v[6:9], v54, s[40:43], 0 offen sc0 sc1
	s_nop 1
	v_max3_f32 v6, v31, v32, v33
"""
    bad = isa_check.store_data_hazards(text)
    assert len(bad) == 1 and bad[0][3] == 0 and "v[2:5]" in bad[0][1]


def test_hot_kernels_use_no_private_memory(sqlib):
    """The raw and frame instances of the 256-wide fused kernel and of the
    per-step kernel keep their state in registers: round 4's frame fold first
    put the 360-byte argument block (then a 24-byte override pair whose stores
    the compiler had merged) in private memory, and the frame launches ran 4x
    slower.  The wide-row instances with a 6-wave budget are allowed their
    documented small spills."""
    from stochquant_amd import isa_check
    md = isa_check.kernel_metadata(os.path.join(ROOT, "stochquant_amd", "lib", "libstochquant.so"))
    hot = {k: v for k, v in md.items()
           if ("phi4_tb2_kernelILb1ELb0E" in k or "phi4_tb2p_kernelILb1ELb0E" in k
               or "phi4_step_kernelILi64ELi1ELi1E" in k)}
    assert len(hot) >= 8, sorted(md)[:20]
    bad = {k: v for k, v in hot.items() if v.get("private", 0) != 0}
    assert bad == {}, bad

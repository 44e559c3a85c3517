"""Static check of the built gfx950 code object for the store-data overwrite
hazard.

A 12- or 16-byte VMEM store reads its data VGPRs after issue; a VALU write of
one of them within two wait states can land first.  On gfx950 the compiler
pads that with `s_nop 1` -- except for buffer stores whose soffset is an SGPR
(GCNHazardRecognizer::createsVALUHazard treats those as hazard-free), and the
frame kernels of round 2's one-accumulator variant stored wrong first
components from exactly that pattern.  The kernels now keep soffset at 0; this
module disassembles libstochquant.so's device code and lists every store of
more than 8 bytes followed, within two wait states, by a VALU write of its data
registers.  Used by tests/test_isa_hazards.py (CPU only: it reads the ELF).
"""
import os
import re
import subprocess
import tempfile

LLVM = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "llvm", "bin")
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
STORE = re.compile(r"(buffer|global|flat|scratch)_store_(dwordx3|dwordx4|b96|b128)\b")
FUNC = re.compile(r"^[0-9a-f]+ <(\S+)>:")


def _regs(tok):
    out = set()
    for m in re.finditer(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b", tok):
        if m.group(3):
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def disassemble(lib):
    """Device code of `lib` (a host .so / .o with a .hip_fatbin), as llvm-objdump text."""
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "k.co")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", lib,
                        os.path.join(d, "x.o")], check=True, capture_output=True)
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fat}",
                        f"--targets={TARGET}", f"--output={co}"], check=True, capture_output=True)
        return subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", co], check=True,
                              capture_output=True, text=True).stdout


def store_data_hazards(text, wait_states=2):
    """[(function, store, overwriting instruction, wait states between)]."""
    ins, fn = [], None
    for line in text.split("\n"):
        m = FUNC.match(line.strip())
        if m:
            fn = m.group(1)
            continue
        t = line.split("//")[0].strip()
        if t and not t.startswith((";", ".")) and not t.endswith(":"):
            ins.append((fn, t))
    found = []
    for i, (f, t) in enumerate(ins):
        op = t.split()[0]
        if not STORE.match(op):
            continue
        parts = t.split(None, 1)[1].split(",")
        data = _regs(parts[0] if op.startswith("buffer") else parts[1])
        ws = 0
        for g, u in ins[i + 1:i + 8]:
            if g != f or ws >= wait_states:
                break
            o2 = u.split()[0]
            if o2 == "s_nop":
                ws += int(u.split()[1], 0) + 1
                continue
            if o2.startswith("v_") and not o2.startswith(("v_readlane", "v_readfirstlane", "v_cmp")):
                if _regs(u.split(None, 1)[1].split(",")[0]) & data:
                    found.append((f, t, u, ws))
                    break
            ws += 1
    return found


def kernel_metadata(lib):
    """{kernel name: {"private": private_segment_fixed_size, "vgpr": vgpr_count,
    "vgpr_spill": vgpr_spill_count}} from the code object's AMDGPU metadata."""
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "k.co")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", lib,
                        os.path.join(d, "x.o")], check=True, capture_output=True)
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fat}",
                        f"--targets={TARGET}", f"--output={co}"], check=True, capture_output=True)
        text = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True, capture_output=True,
                              text=True).stdout
    out = {}
    for block in text.split("    .name:")[1:]:
        name = block.split()[0]
        rec = {}
        for key, field in (("private", ".private_segment_fixed_size"), ("vgpr", ".vgpr_count"),
                           ("vgpr_spill", ".vgpr_spill_count")):
            m = re.search(re.escape(field) + r":\s+(\d+)", block)
            if m:
                rec[key] = int(m.group(1))
        out[name] = rec
    return out

"""Code-object checks on the built libraries (CPU only, no GPU): the gfx950
code object is present, no kernel uses scratch, and the hot kernel's loads
are global (not flat) non-temporal 16-B loads."""
import os
import re
import shutil
import subprocess

import pytest

from conftest import ROOT

LLVM = "/opt/rocm/lib/llvm/bin"
LIBS = [os.path.join(ROOT, "feddct_amd", "libfedagg.so"),
        os.path.join(ROOT, "feddct_amd", "libfedagg_comm.so")]
HOT = "_ZN12_GLOBAL__N_113reduce_kernelILi2ELi16ELb0ELb0ELi3ELb0EEEvNS_10ReduceArgsE"


def _have_tools():
    return all(os.path.exists(os.path.join(LLVM, t))
               for t in ("clang-offload-bundler", "llvm-objdump", "llvm-readelf")) and \
        shutil.which("objcopy")


def _code_object(lib, tmp_path):
    fb = tmp_path / (os.path.basename(lib) + ".fatbin")
    co = tmp_path / (os.path.basename(lib) + ".co")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, str(fb)],
                   check=True)
    targets = subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--list", "--type=o",
                              f"--input={fb}"], check=True, capture_output=True,
                             text=True).stdout.split()
    assert "hipv4-amdgcn-amd-amdhsa--gfx950" in targets, targets
    subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                    f"--input={fb}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                    f"--output={co}"], check=True)
    return str(co)


def _kernels(co):
    notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True,
                           capture_output=True, text=True).stdout
    out, cur = {}, None
    for line in notes.splitlines():
        m = re.match(r"\s+\.name:\s+(\S+)", line)
        if m:
            cur = m.group(1)
        m = re.match(r"\s+\.private_segment_fixed_size:\s+(\d+)", line)
        if m and cur is not None:
            out[cur] = int(m.group(1))
    return out


@pytest.mark.skipif(not _have_tools(), reason="ROCm llvm tools / objcopy not available")
@pytest.mark.parametrize("lib", LIBS)
def test_code_object_has_gfx950_and_no_scratch(lib, tmp_path):
    co = _code_object(lib, tmp_path)
    kernels = _kernels(co)
    assert kernels, "no kernels found in the code object"
    assert {k: v for k, v in kernels.items() if v} == {}, "kernels using scratch"


@pytest.mark.skipif(not _have_tools(), reason="ROCm llvm tools / objcopy not available")
def test_hot_kernel_uses_global_nt_loads(tmp_path):
    co = _code_object(LIBS[0], tmp_path)
    dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", co], check=True,
                         capture_output=True, text=True).stdout
    m = re.search(re.escape(HOT) + r">:\n(.*?)\n\n", dis, flags=re.S)
    assert m, "default reduce kernel not found"
    body = m.group(1)
    loads = re.findall(r"\b(global|flat|buffer)_load_dwordx4\b[^\n]*", body)
    assert loads and not re.search(r"\bflat_load_dwordx4\b", body), "hot loads are flat"
    nt = re.findall(r"global_load_dwordx4[^\n]*\bnt\b", body)
    assert len(nt) >= 32, "hot loads should be non-temporal global_load_dwordx4"
    assert "scratch_" not in body

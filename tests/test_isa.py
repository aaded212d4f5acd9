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
HOT = "_ZN4fa_k13reduce_kernelILi2ELi16ELb0ELb0ELi3ELb0EEEvNS_10ReduceArgsE"


def _have_tools():
    return all(os.path.exists(os.path.join(LLVM, t))
               for t in ("clang-offload-bundler", "llvm-objdump", "llvm-readelf")) and \
        shutil.which("objcopy")


MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _code_objects(lib, tmp_path):
    """The gfx950 code object of every translation unit: the .hip_fatbin
    section holds one offload bundle per unit (libfedagg.so is built from
    several, feddct_amd/build.py), each starting with the bundle magic."""
    fb = tmp_path / (os.path.basename(lib) + ".fatbin")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, str(fb)],
                   check=True)
    data = fb.read_bytes()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    assert starts, "no offload bundle in " + lib
    cos = []
    for k, (a, b) in enumerate(zip(starts, starts[1:] + [len(data)])):
        part = tmp_path / f"{os.path.basename(lib)}.{k}.bundle"
        part.write_bytes(data[a:b])
        co = tmp_path / f"{os.path.basename(lib)}.{k}.co"
        targets = subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--list",
                                  "--type=o", f"--input={part}"], check=True,
                                 capture_output=True, text=True).stdout.split()
        assert "hipv4-amdgcn-amd-amdhsa--gfx950" in targets, targets
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                        f"--input={part}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        f"--output={co}"], check=True)
        cos.append(str(co))
    return cos


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
    kernels = {}
    for co in _code_objects(lib, tmp_path):
        kernels.update(_kernels(co))
    assert kernels, "no kernels found in the code objects"
    assert {k: v for k, v in kernels.items() if v} == {}, "kernels using scratch"


@pytest.mark.skipif(not _have_tools(), reason="ROCm llvm tools / objcopy not available")
def test_every_reduce_variant_is_compiled_once(tmp_path):
    """The reduce kernel family is split over several units (build.py); no
    instance may be compiled in two of them (each unit registers its own
    code object for the kernels it launches)."""
    seen = {}
    for k, co in enumerate(_code_objects(LIBS[0], tmp_path)):
        for name in _kernels(co):
            assert name not in seen, (name, seen.get(name), k)
            seen[name] = k
    assert HOT in seen


@pytest.mark.skipif(not _have_tools(), reason="ROCm llvm tools / objcopy not available")
def test_hot_kernel_uses_global_nt_loads(tmp_path):
    body = None
    for co in _code_objects(LIBS[0], tmp_path):
        dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", co], check=True,
                             capture_output=True, text=True).stdout
        m = re.search(re.escape(HOT) + r">:\n(.*?)(?:\n\n|\Z)", dis, flags=re.S)
        if m:
            body = m.group(1)
    assert body, "default reduce kernel not found"
    loads = re.findall(r"\b(global|flat|buffer)_load_dwordx4\b[^\n]*", body)
    assert loads and not re.search(r"\bflat_load_dwordx4\b", body), "hot loads are flat"
    nt = re.findall(r"global_load_dwordx4[^\n]*\bnt\b", body)
    assert len(nt) >= 32, "hot loads should be non-temporal global_load_dwordx4"
    assert "scratch_" not in body

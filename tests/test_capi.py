"""The drop-in boundary: libhecdna.so loads (no GPU needed) and exports every symbol that
include/hecdna.h declares; no compute calls here."""
import ctypes
import subprocess


def test_header_symbols_exported(hecdna):
    declared = hecdna.exported_symbols()
    assert len(declared) >= 50
    out = subprocess.check_output(["nm", "-D", "--defined-only", hecdna.LIB_PATH]).decode()
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [s for s in declared if s not in exported]
    assert not missing, missing


def test_library_loads_and_binds(hecdna):
    L = hecdna.lib()
    assert L.hec_version() >= 100
    assert isinstance(L.hec_last_error(), bytes)


def test_no_torch_types_in_boundary(hecdna):
    txt = open(hecdna.HEADER_PATH).read()
    assert "torch" not in txt.replace("No torch types cross this boundary", "")
    assert 'extern "C"' in txt


def test_product_does_not_reference_oracle(hecdna):
    import os
    pkg = os.path.dirname(hecdna.LIB_PATH)
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".hip", ".h", ".py", ".cpp", ".hpp")):
                src = open(os.path.join(root, f)).read()
                assert "oracle" not in src.lower(), f
    syms = subprocess.check_output(["nm", "-D", hecdna.LIB_PATH]).decode()
    assert "orc_" not in syms


def test_host_logic_without_gpu(hecdna):
    # pure host entry points work without a device
    m = hecdna.create_coeff_modulus(1 << 13, [60, 40, 40, 60])
    assert m == [0xffffffffffe8001, 0xfffff4c001, 0xfffffdc001, 0xfffffffffffc001]
    with __import__("pytest").raises(hecdna.InvalidArgument):
        hecdna.create_coeff_modulus(1000, [60])
    assert ctypes.sizeof(ctypes.c_void_p) == 8


def test_cpp_facade_links_against_boundary(hecdna, tmp_path):
    """The C++ drop-in headers (he_operators.h / he_linalg.h over hecdna types) compile and the
    demo links against libhecdna.so using only the C-ABI."""
    import os
    pkg = os.path.dirname(hecdna.LIB_PATH)
    exe = str(tmp_path / "he_demo")
    subprocess.check_call(["g++", "-std=c++20", "-O0", "-I" + os.path.join(pkg, "cpp", "include"),
                           "-I" + os.path.join(pkg, "..", "include"),
                           os.path.join(pkg, "cpp", "demo", "he_demo.cpp"),
                           os.path.join(pkg, "cpp", "src", "he_operators.cpp"),
                           os.path.join(pkg, "cpp", "src", "he_linalg.cpp"), os.path.join(pkg, "cpp", "src", "he_math.cpp"),
                           "-L" + pkg, "-lhecdna", "-o", exe])
    out = subprocess.run([exe], capture_output=True, text=True, env=dict(os.environ, LD_LIBRARY_PATH=pkg))
    assert out.returncode == 1 and "usage" in out.stdout

"""CPU checks of the C ABI library: it loads, and exports every symbol
include/*.h declares (no compute calls -- there is no GPU here)."""
import ctypes
import os
import re

from oracle import evolu_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    import glob

    text = "".join(open(h).read() for h in sorted(glob.glob(os.path.join(ROOT, "include", "*.h"))))
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(evm_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from evolu_amd import _lib, build

    build.build_lib()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    # the ctypes binding covers the header exactly
    assert sorted(_lib.SIGNATURES) == syms
    assert lib.evm_strerror.restype is not None or True


def test_strerror_no_gpu_needed():
    from evolu_amd import _lib

    lib = _lib.load()
    assert lib.evm_strerror(0) == b"ok"
    assert b"RangeError" in lib.evm_strerror(4)


def test_minute_arithmetic_matches_js_on_native_range():
    # merkleTree.ts:33 (millis/1000/60)|0 == floor(millis/60000) for 0 <= millis < 2^31 minutes
    import random

    r = random.Random(3)
    for k in list(range(0, 2**31, 99991)) + [2**31 - 1]:
        for d in (-1, 0, 1):
            m = k * 60000 + d
            if 0 <= m < 2**31 * 60000:
                assert O.to_int32(m / 1000 / 60) == m // 60000
    for _ in range(20000):
        m = r.randrange(0, 2**31 * 60000)
        assert O.to_int32(m / 1000 / 60) == m // 60000


def test_dist_unique_id_without_gpu():
    """evm_dist_unique_id needs RCCL's bootstrap only (no device)."""
    from evolu_amd.engine import dist_unique_id

    a, b = dist_unique_id(), dist_unique_id()
    assert len(a) == 128 and a != b


def test_device_code_has_no_floating_point():
    """Every kernel of libevm is integer work (exact integer /
    bitwise arithmetic).  A double instruction in the device code means some
    min / max of a 64-bit key resolved to HIP's double overload (a mixed
    unsigned long / unsigned long long pair does) and drops the low bits of
    millis << 16 | counter -- the bug that once made K5's max miss a
    counter.  Disassembles the built gfx950 code objects (no GPU needed)."""
    import glob
    import os
    import shutil
    import subprocess
    import tempfile

    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if not os.path.exists(objdump):
        pytest.skip("llvm-objdump not present")
    from evolu_amd import _lib

    with tempfile.TemporaryDirectory() as d:
        lib = os.path.join(d, "libevm.so")
        shutil.copy(_lib.LIB_PATH, lib)
        subprocess.run([objdump, "--offloading", lib], check=True, capture_output=True, cwd=d)
        objs = glob.glob(os.path.join(d, "libevm.so.*gfx950"))
        assert objs
        for o in objs:
            asm = subprocess.run([objdump, "-d", "--mcpu=gfx950", o], check=True, capture_output=True,
                                 text=True).stdout
            # (f32 ops are the compiler's expansion of 32-bit integer division: exact)
            bad = [ln for ln in asm.splitlines() if "_f64" in ln]
            assert not bad, bad[:5]

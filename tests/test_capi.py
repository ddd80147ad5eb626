"""CPU: the C-ABI library loads and exports every symbol include/roce_icrc.h
declares; without a GPU the product fails loudly (no CPU fallback)."""
import ctypes

import pytest

from roce_icrc import engine as E


def test_library_exports_every_header_symbol():
    lib = E.load_library()
    names = E.header_functions()
    assert len(names) >= 20
    for name in names:
        assert hasattr(lib, name), name
    # the ctypes signature table covers the header exactly
    assert set(E._SIGNATURES) == set(names)


def test_abi_version_and_errors():
    lib = E.load_library()
    assert lib.ricrc_abi_version() == 5
    assert lib.ricrc_strerror(0) == b"ok"
    assert lib.ricrc_strerror(-22) == b"invalid argument"
    assert lib.ricrc_strerror(-19) == b"no usable gfx950 device"


def test_null_arguments_rejected_without_touching_a_device():
    lib = E.load_library()
    assert lib.ricrc_ctx_create(0, None) == -22
    assert lib.ricrc_compute_one(None, None, 0, None, None) == -22
    assert lib.ricrc_icrc(None, 0, None, None) == -22
    assert lib.ricrc_compute_batch_multi(None, 0, None, 0, None, None, 0, None, None) == -22
    assert lib.ricrc_verify_batch_multi(None, 0, None, 0, None, None, 0, None, None, None) == -22
    assert lib.ricrc_ctx_set_lanes_per_packet(None, 8) == -22


def test_no_gpu_means_no_engine():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible here")
    assert E.device_count() == 0
    with pytest.raises(E.IcrcUnavailable):
        E.IcrcEngine(0)
    # the context-free call finds no device either (no CPU fallback)
    with pytest.raises(E.IcrcError) as ei:
        E.icrc(b"\x45" + bytes(59))
    assert ei.value.code == -19


def test_product_package_never_imports_the_oracle():
    import pathlib
    pkg = pathlib.Path(E.__file__).parent
    for f in list(pkg.glob("*.py")) + list((pkg.parent / "csrc").glob("*")):
        text = f.read_text(errors="ignore")
        assert "icrc_oracle" not in text and "liboracle" not in text, f


def build_abi_consumer(tmp_path):
    """Compile tests/c/abi_consumer.c as C99 against include/roce_icrc.h and
    link it to the library (also used by the GPU run in test_gpu_capi.py)."""
    import shutil
    import subprocess
    from pathlib import Path
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    root = Path(__file__).resolve().parent.parent
    lib = E.library_path()
    exe = tmp_path / "abi_consumer"
    subprocess.run([cc, "-std=c99", "-Wall", "-Werror", "-I", str(root / "include"),
                    str(root / "tests" / "c" / "abi_consumer.c"), "-L", str(lib.parent),
                    "-l:" + lib.name, "-Wl,-rpath," + str(lib.parent), "-o", str(exe)],
                   check=True)
    return exe


def test_header_is_plain_c_and_links(tmp_path):
    """include/roce_icrc.h compiles as C99 and a C program links the library
    and calls it (no GPU here: planning, errors, ENODEV without a device; the
    GPU run of the same program is tests/test_gpu_capi.py)."""
    import subprocess
    exe = build_abi_consumer(tmp_path)
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU visible: the run leg is tests/test_gpu_capi.py")
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    assert out.startswith("abi 5 ok: 4 packets, slot 4224"), out
    assert "gpu leg skipped" in out


def test_descriptor_arrays_must_match():
    """offsets and lens of a ragged batch must have one entry per frame each
    (a shorter lens array would make the C library read past its end)."""
    import numpy as np
    offs, ls = E._descriptors([0, 64, 128], [44, 44, 44])
    assert offs.dtype == np.uint64 and ls.dtype == np.uint32
    with pytest.raises(ValueError):
        E._descriptors([0, 64, 128], [44, 44])
    with pytest.raises(ValueError):
        E._descriptors(np.zeros((2, 2)), np.zeros((2, 2)))


def test_pack_aligned_keeps_every_frame_dword_aligned():
    import numpy as np
    frames = [b"\x01" * 47, b"\x02" * 3, b"\x03" * 44, b"", b"\x04" * 5]
    buf, offs, lens = E.pack_aligned(frames)
    assert list(lens) == [47, 3, 44, 0, 5]
    assert list(offs) == [0, 48, 52, 96, 96]
    assert (offs % 4 == 0).all() and buf.size == 104
    for f, o in zip(frames, offs):
        assert buf[int(o):int(o) + len(f)].tobytes() == f

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
    assert lib.ricrc_abi_version() == 2
    assert lib.ricrc_strerror(0) == b"ok"
    assert lib.ricrc_strerror(-22) == b"invalid argument"
    assert lib.ricrc_strerror(-19) == b"no usable gfx950 device"


def test_null_arguments_rejected_without_touching_a_device():
    lib = E.load_library()
    assert lib.ricrc_ctx_create(0, None) == -22
    assert lib.ricrc_compute_one(None, None, 0, None, None) == -22
    assert lib.ricrc_compute_batch_multi(None, 0, None, 0, None, None, 0, None, None) == -22
    assert lib.ricrc_ctx_set_lanes_per_packet(None, 8) == -22


def test_no_gpu_means_no_engine():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible here")
    assert E.device_count() == 0
    with pytest.raises(E.IcrcUnavailable):
        E.IcrcEngine(0)


def test_product_package_never_imports_the_oracle():
    import pathlib
    pkg = pathlib.Path(E.__file__).parent
    for f in list(pkg.glob("*.py")) + list((pkg.parent / "csrc").glob("*")):
        text = f.read_text(errors="ignore")
        assert "icrc_oracle" not in text and "liboracle" not in text, f


def test_header_is_plain_c_and_links(tmp_path):
    """include/roce_icrc.h compiles as C99 and a C program links the library
    and calls it (no GPU needed: planning, errors, ENODEV without a device)."""
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
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("the run leg is for GPU-less hosts (device 0 would be initialised)")
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    assert out.startswith("abi 2 ok: 4 packets, slot 4352"), out

"""CPU: the C-ABI library loads and exports exactly what include/scflow_hip.h declares."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "scflow_hip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(scflow_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_path():
    names = declared_functions()
    for must in ("scflow_corr_pyramid", "scflow_corr_lookup", "scflow_conv2d",
                 "scflow_pose_update_flow", "scflow_lift_points", "scflow_flow_downsample",
                 "scflow_flow_upsample"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from scflow_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        from scflow_amd import build
        build.build()
    lib = _lib.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
        assert name in _lib.SIGNATURES, f"{name} has no ctypes signature"
    assert lib.scflow_version() >= 1
    assert lib.scflow_strerror(-2).decode().startswith("unsupported")


def test_host_side_queries_need_no_gpu():
    from scflow_amd import _lib
    lib = _lib.load()
    # pyramid size: 16 pairs, 32×32, 4 levels = 16·1024·(1024+256+64+16)
    assert lib.scflow_corr_pyramid_size(16, 32, 32, 4) == 16 * 1024 * 1360
    # conv packing geometry: GRU z|r (256 out, 384 in, 1×5): 256 × 5·384
    assert lib.scflow_conv_packed_size(256, 384, 0, 1, 5, 1, 32) == 256 * 5 * 384
    # cin 324 is padded to 336 per tap; cout 126 to 128
    assert lib.scflow_conv_packed_size(126, 324, 0, 1, 1, 1, 32) == 128 * 336
    assert lib.scflow_conv_packed_size(64, 64, 0, 3, 3, 1, 20) < 0  # width not tileable → unsupported
    # Winograd packing: 16 transform points × cout padded to 64 × cin padded to 32 per source
    assert lib.scflow_conv_packed_size_bk(192, 256, 0, 3, 3, 1, 32, 2) == 16 * 192 * 256
    assert lib.scflow_conv_packed_size_bk(126, 192, 60, 3, 3, 1, 32, 2) == 16 * 128 * (192 + 64)
    # F(4,5) packing: 8 transform points × cout padded to 64 × cin padded to 32 per source
    assert lib.scflow_conv_packed_size_bk(64, 64, 0, 1, 5, 1, 32, 2) == 8 * 64 * 64
    assert lib.scflow_conv_packed_size_bk(128, 120, 8, 5, 1, 1, 32, 2) == 8 * 128 * (128 + 32)
    assert lib.scflow_conv_packed_size_bk(64, 64, 0, 1, 1, 1, 32, 2) < 0  # 3×3 / 1×5 / 5×1 only
    assert lib.scflow_conv_packed_size_bk(64, 64, 0, 3, 3, 1, 32, 16) == 64 * 64 * 9
    # argument errors return codes, they do not crash
    assert lib.scflow_corr_pyramid(None, None, None, 1, 1, 8, 8, 4, None) == -1
    assert lib.scflow_conv2d(None, None) == -1
    # encoder conv packing: 3×3 96→96 (cout padded to 128), stem 7×7·3 → 64
    assert lib.scflow_enc_conv_packed_size(96, 96, 3, 3) == 128 * 96 * 9
    assert lib.scflow_enc_stem_packed_size(64, 3, 7, 7) == 147 * 64
    assert lib.scflow_enc_conv(None, None) == -1


@pytest.mark.parametrize("pyname,cname", [("ConvArgs", "scflow_conv_args"),
                                           ("EncConvArgs", "scflow_enc_conv_args"),
                                           ("WgradArgs", "scflow_wgrad_args"),
                                           ("RenderArgs", "scflow_render_args")])
def test_struct_layout_matches_header(tmp_path, pyname, cname):
    """ctypes argument structs have the C compiler's size and field offsets."""
    import shutil
    import subprocess
    from scflow_amd import _lib
    S = getattr(_lib, pyname)
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    fields = [f for f, _ in S._fields_]
    prog = tmp_path / "layout.c"
    prog.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "scflow_hip.h"\nint main(){\n'
                    f'printf("%zu\\n", sizeof({cname}));\n' +
                    "".join(f'printf("%zu\\n", offsetof({cname}, {f}));\n' for f in fields) +
                    "return 0;}\n")
    exe = tmp_path / "layout"
    subprocess.run([cc, "-I", os.path.join(ROOT, "include"), str(prog), "-o", str(exe)], check=True)
    vals = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True,
                                           check=True).stdout.split()]
    assert vals[0] == ctypes.sizeof(S)
    for f, off in zip(fields, vals[1:]):
        assert getattr(S, f).offset == off, f

"""The C-ABI library loads and exports every symbol include/qlzx.h declares (no GPU)."""
import ctypes
import os
import subprocess

from gobeansdb_amd import _lib, build


def test_library_builds_and_exports_header_symbols():
    build.build()
    L = _lib.lib()
    names = _lib.header_functions()
    assert {"qlz_compress", "qlz_decompress", "qlz_size_compressed", "qlz_size_decompressed",
            "qlz_get_setting", "crc32_write", "qlzx_decompress_batch", "qlzx_compress_batch",
            "qlzx_crc32_batch"} <= set(names)
    for n in names:
        assert hasattr(L, n), n
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert set(names) <= exported


def test_gfx950_code_object_present(tmp_path):
    # the fat binary section (.hip_fatbin) holds one zstd-compressed offload bundle ("CCOB") per
    # translation unit (qlzx_api.hip and qlzx_k2.hip since round 5): each carries a gfx950 code
    # object -- list every bundle's entries with the ROCm LLVM tools
    import re
    bin_dir = "/opt/rocm/lib/llvm/bin"
    fb = tmp_path / "fatbin.bin"
    subprocess.run([f"{bin_dir}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", _lib.LIB_PATH,
                    str(tmp_path / "host.o")], check=True)
    data = fb.read_bytes()
    starts = [m.start() for m in re.finditer(b"CCOB|__CLANG_OFFLOAD_BUNDLE__", data)]
    assert starts and starts[0] == 0
    import struct
    for a, b in zip(starts, starts[1:] + [len(data)]):
        end = b
        if data[a:a + 4] == b"CCOB":  # compressed bundle: its header holds its total size (v3: u64, v2: u32)
            ver = struct.unpack_from("<H", data, a + 4)[0]
            end = a + (struct.unpack_from("<Q", data, a + 8)[0] if ver >= 3 else struct.unpack_from("<I", data, a + 8)[0])
        part = tmp_path / f"bundle_{a}.bin"
        part.write_bytes(data[a:end])
        out = subprocess.run([f"{bin_dir}/clang-offload-bundler", "--list", "--type=o", f"--input={part}"],
                             capture_output=True, text=True, check=True).stdout
        assert "hipv4-amdgcn-amd-amdhsa--gfx950" in out.split(), (a, out)


def test_settings_match_reference(golden):
    L = _lib.lib()
    for k, v in golden.manifest["settings"].items():
        assert L.qlz_get_setting(int(k)) == v


def test_header_helpers(golden):
    L = _lib.lib()
    for v in golden.vectors:
        c = golden.get(v["c_out"])
        buf = ctypes.create_string_buffer(c, max(len(c), 9))
        assert L.qlz_size_compressed(buf) == len(c)
        assert L.qlz_size_decompressed(buf) == v["n"]


def test_info_names_gfx950():
    assert "gfx950" in _lib.info()


def test_library_built_from_this_tree():
    """The shipped libqlzx.so carries the hash of the sources it was compiled from
    (build.source_hash over csrc/* + include/qlzx.h), and it is this tree's."""
    _lib.lib()
    h = build.source_hash()
    assert build.embedded_hash() == h
    assert ("src " + h) in _lib.info()


def test_drop_ins_fail_stop_without_a_device():
    """The quicklz.h drop-ins have no error channel in their Go callers
    (quicklz/cquicklz.go:38-40, store/crc32.go:81-84): on a host with no GPU, qlz_compress,
    qlz_decompress and crc32_write must stop the process with the reason, not return 0 (an
    empty "compressed" value) or the input CRC state (a plausible wrong record CRC)."""
    import sys
    build.build()
    for call in ("L.qlz_compress(b'abcdefgh' * 64, ctypes.create_string_buffer(1024), 512, None)",
                 "L.qlz_decompress(bytes([0x4d, 12, 3]) + bytes(9), ctypes.create_string_buffer(64), None)",
                 "L.crc32_write(0xffffffff, b'abc', 3)"):
        code = ("import ctypes, sys; sys.path.insert(0, %r); from gobeansdb_amd import _lib; "
                "L = _lib.lib(); r = %s; print('returned', r)") % (os.path.dirname(os.path.dirname(__file__)), call)
        env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
        p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
        assert p.returncode != 0, (call, p.stdout, p.stderr)
        assert "returned" not in p.stdout
        assert "libqlzx:" in p.stderr and "no error channel" in p.stderr, p.stderr


def test_service_test_hook_is_inert_by_default():
    """qlzx_service_test_fault is a test hook: without QLZX_TEST_HOOKS=1 in the process
    environment it refuses (QLZX_R_BAD_ARG = -1) before touching the request service, so no caller
    of the release library can make another thread's drop-in call fail."""
    import sys
    code = ("import sys; sys.path.insert(0, %r); from gobeansdb_amd import _lib; "
            "L = _lib.lib(); print('rc', L.qlzx_service_test_fault(1)); "
            "print('err', L.qlzx_last_error().decode())") % (os.path.dirname(os.path.dirname(__file__)),)
    env = {k: v for k, v in os.environ.items() if k != "QLZX_TEST_HOOKS"}
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    assert p.returncode == 0, p.stderr
    assert "rc -1" in p.stdout and "test hooks are off" in p.stdout, p.stdout

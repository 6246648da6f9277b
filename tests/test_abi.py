"""The C-ABI boundary without a GPU: the library loads, exports every symbol
include/hip_crc32c_batch.h declares, validates arguments, and the C++ drop-in
surface (include/wipdb/crc32c.h) compiles and passes the reference's tests."""
import ctypes
import os
import subprocess

import pytest

from wipdb_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    syms = _lib.header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    # and every prototype the binding declares is in the header
    assert set(_lib._PROTOS) == set(syms)


def test_header_flag_values_match_binding():
    """Every HCRC_* value macro of include/hip_crc32c_batch.h that the
    Python binding names (flags such as HCRC_BALANCE, error codes) has the
    header's value."""
    import re
    hdr = open(os.path.join(REPO, "include", "hip_crc32c_batch.h")).read()
    macros = {m.group(1): int(m.group(2), 0) for m in
              re.finditer(r"#define (HCRC_[A-Z_]+) \(?(-?(?:0x)?[0-9A-Fa-f]+)\)?", hdr)}
    named = {k: getattr(_lib, k) for k in macros if hasattr(_lib, k)}
    assert {"HCRC_DEVICE_PTRS", "HCRC_SPLIT_SMALL", "HCRC_SPLIT_LONG", "HCRC_BALANCE",
            "HCRC_PACKED"} <= set(named)
    for k, v in named.items():
        assert v == macros[k], (k, v, macros[k])


def test_abi_version_and_strerror():
    lib = _lib.load()
    assert lib.hcrc_abi_version() == 1
    for code in (0, -1, -2, -3, -4, -5, -6, -7, -99):
        assert lib.hcrc_strerror(code)


def test_invalid_arguments_are_rejected_without_device():
    lib = _lib.load()
    assert lib.hcrc_ctx_create(0, None) == _lib.HCRC_ERR_INVALID
    assert lib.hcrc_ctx_shared(0, None) == _lib.HCRC_ERR_INVALID
    assert lib.hcrc_ctx_destroy(None) == _lib.HCRC_ERR_INVALID
    assert lib.hcrc_batch(None, None, None, None, None, None, 0, 0) == _lib.HCRC_ERR_INVALID
    assert lib.hcrc_batch_async(None, None, None, None, None, None, 0, 1, None) == _lib.HCRC_ERR_INVALID
    assert lib.hcrc_sync(None, None) == _lib.HCRC_ERR_INVALID
    assert lib.hcrc_check_spans(None, 0, None, None, 0, 0, None) == _lib.HCRC_ERR_INVALID
    assert lib.hcrc_check_spans_async(None, 0, None, None, 0, 0, None, None) == _lib.HCRC_ERR_INVALID
    devs = (ctypes.c_int * 1)(0)
    assert lib.hcrc_batch_multi(devs, 0, None, None, None, None, None, 0, 0) == _lib.HCRC_ERR_INVALID
    assert lib.hcrc_cpu_batch(None, None, None, None, None, 1, 0, 1) == _lib.HCRC_ERR_INVALID
    n = ctypes.c_int(-1)
    rc = lib.hcrc_device_count(ctypes.byref(n))
    assert (rc == 0 and n.value >= 0) or (rc == _lib.HCRC_ERR_NO_DEVICE and n.value == 0)


def test_host_memory_entry_points_validate_arguments():
    lib = _lib.load()
    assert lib.hcrc_host_register(None, 4096) == _lib.HCRC_ERR_INVALID
    assert lib.hcrc_host_register(1, 0) == _lib.HCRC_ERR_INVALID
    assert lib.hcrc_host_unregister(None) == _lib.HCRC_ERR_INVALID
    assert lib.hcrc_host_alloc(16, None) == _lib.HCRC_ERR_INVALID


def test_ctx_create_bad_device_index():
    lib = _lib.load()
    ctx = ctypes.c_void_p()
    assert lib.hcrc_ctx_create(10_000, ctypes.byref(ctx)) == _lib.HCRC_ERR_NO_DEVICE
    assert not ctx.value


def _build_surface_test(tmp_path):
    exe = str(tmp_path / "test_surface")
    libdir = os.path.join(REPO, "wipdb_amd", "lib")
    cmd = ["g++", "-O2", "-std=c++17", "-I", os.path.join(REPO, "include"),
           "-I", os.path.join(REPO, "include", "wipdb_compat"),
           os.path.join(REPO, "tests", "cpp", "test_surface.cc"), "-L", libdir,
           "-lhip_crc32c_batch", f"-Wl,-rpath,{libdir}", "-o", exe]
    subprocess.run(cmd, check=True)
    return exe


def test_cpp_surface_drop_in_cpu(tmp_path):
    from tests.conftest import gpu_available
    if gpu_available():
        pytest.skip("GPU present: covered by tests/test_gpu_parity.py::test_cpp_surface_drop_in_gpu")
    exe = _build_surface_test(tmp_path)
    r = subprocess.run([exe, "0"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS" in r.stdout
    # the runtime selector: WIPDB_CRC_MODE=cpu, a device list, a threshold --
    # without a device every kAuto batch still lands on the host
    env = dict(os.environ, WIPDB_CRC_MODE="cpu", WIPDB_CRC_DEVICES="0,1",
               WIPDB_CRC_MIN_GPU_BATCH="1")
    r = subprocess.run([exe, "0"], capture_output=True, text=True, env=env)
    assert r.returncode == 0, r.stdout + r.stderr


def test_kernel_span_geometry_host(tmp_path):
    """tests/cpp/test_walk.cc: the LDS kernels' span geometry
    (wipdb_amd/csrc/crc32c_walk.h) on the host -- every DMA source of every
    span shape stays in the span's pages, and replaying the kernel's
    arithmetic on those sources gives Extend() and ReadBlock's verdict for
    84 k (start, length, init, verify) cases."""
    exe = str(tmp_path / "test_walk")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(REPO, "wipdb_amd", "csrc"),
                    os.path.join(REPO, "tests", "cpp", "test_walk.cc"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "PASS" in r.stdout


def test_lane_packed_plan_host(tmp_path):
    """tests/cpp/test_plan.cc: the lane-packed kernels' span plans
    (wipdb_amd/csrc/crc32c_plan.h) on the host -- segments from the start,
    the back piece's lanes and stripes as the batch DMA derives them: every
    DMA source dword-aligned and in the span's pages, and the kernel's
    arithmetic replayed on those sources (zeroed in-front chunks, injected
    registers, per-lane shifts, the tail from the aux chunk) gives Extend()
    and ReadBlock's verdict for ~87 k (start, length, init, verify) cases."""
    exe = str(tmp_path / "test_plan")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(REPO, "wipdb_amd", "csrc"),
                    os.path.join(REPO, "tests", "cpp", "test_plan.cc"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "PASS" in r.stdout


def test_lane_packed_kernels_emulated(tmp_path):
    """tests/cpp/test_lp_emu.cc: the spans / verify / strided kernels' own
    source (wipdb_amd/csrc/crc32c_lds.hip) compiled for the host against the
    SIMT emulation of their primitives (tests/cpp/lk_emu.h: a thread per
    lane, DPP / ballot / bpermute through per-wave exchanges, LDS and its
    atomics in host memory, DMA copies range-checked), run over every span
    shape (short spans packed per iteration, table blocks, long spans shared
    through the workgroup queue, empties, inits, masks), verify with
    corruptions, and strided blocks -- bit-exact with a byte-serial CRC.
    The launch-level pipeline choice (run_ea for 4 KiB-class and >= 32 KiB
    batches, run_lp otherwise) is checked per shape, and a second run forces
    run_ea on every shape."""
    clang = "/opt/rocm/lib/llvm/bin/clang++"
    if not os.path.exists(clang):
        pytest.skip("ROCm clang++ not present")
    exe = str(tmp_path / "test_lp_emu")
    subprocess.run([clang, "-std=c++20", "-O1", "-pthread", "-Wno-unused-function",
                    "-I", os.path.join(REPO, "wipdb_amd", "csrc"), "-I", os.path.join(REPO, "tests", "cpp"),
                    os.path.join(REPO, "tests", "cpp", "test_lp_emu.cc"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "PASS" in r.stdout
    # the same shapes with every launch forced onto run_ea (the launch's
    # pipeline choice only changes speed: both pipelines must be exact on
    # every shape, whatever the sample picked)
    r = subprocess.run([exe, "--pipe=ea", "one", "17", "tiny", "short", "bucket", "near", "small pieces",
                        "long", "zipf", "verify", "strided", "exact fit packed"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "PASS" in r.stdout
    # verdict r4 item 1: exact-fit batches (every column followed by a guard
    # page; the r04an shape's first and last workgroups are in the default
    # run) with every launch forced onto run_lp as well
    r = subprocess.run([exe, "--pipe=lp", "exact fit packed", "exact fit verify 4 KiB"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "PASS" in r.stdout


def test_host_code_under_sanitizers():
    """the library's host code (CPU CRC path, table / log layers,
    compaction input, C-ABI checks) built with -fsanitize=address,undefined
    (make -C wipdb_amd/csrc sanitize) runs clean over clean and damaged
    inputs (tests/cpp/test_host_sanitize.cc)."""
    from tests.conftest import gpu_available
    if gpu_available():
        pytest.skip("host-only check; run on the CPU container")
    env = dict(os.environ, PYTORCH_ROCM_ARCH="gfx950")
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "wipdb_amd", "csrc"), "sanitize",
                    "ARCH=gfx950"], check=True, env=env, timeout=900)
    exe = os.path.join(REPO, "build", "sanitize", "test_host_sanitize")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
                                UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert "PASS" in r.stdout

"""AddressSanitizer + UndefinedBehaviorSanitizer builds of the host code (no
GPU):

* the C oracle (`make -C oracle asan`, clang) runs the oracle's own test
  files -- the reference fixtures, the sampling-distribution pins and the
  mechanism known answers -- in a child process with the ASan runtime
  preloaded;
* the host side of libdpg (`hipcc --cuda-host-only`, no device code) is
  driven through its C ABI on every entry point's argument-error path and
  through the pure helpers, in a child process with the same runtime.

A sanitizer report aborts the child (halt_on_error), which fails the test.
"""
import glob
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
ASAN_RT = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
ORACLE_ASAN = os.path.join(ROOT, "oracle", "_build", "asan", "libdporacle.so")
DPG_ASAN_DIR = os.path.join(ROOT, "build", "asan")
DPG_ASAN = os.path.join(DPG_ASAN_DIR, "libdpg_asan.so")

pytestmark = pytest.mark.skipif(not ASAN_RT or not os.path.exists(HIPCC),
                                reason="ROCm clang ASan runtime not present")


def _env(**extra):
    env = dict(os.environ)
    env["LD_PRELOAD"] = ASAN_RT[-1]
    env["ASAN_OPTIONS"] = "detect_leaks=0:halt_on_error=1:abort_on_error=1"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    env["PYTHONPATH"] = ROOT
    env.update(extra)
    return env


@pytest.fixture(scope="module")
def oracle_asan():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
    return ORACLE_ASAN


@pytest.fixture(scope="module")
def dpg_asan():
    src = os.path.join(ROOT, "pipelinedp_amd", "csrc")
    deps = glob.glob(os.path.join(src, "*")) + [os.path.join(ROOT, "include", "dpg.h")]
    if not (os.path.exists(DPG_ASAN) and
            os.path.getmtime(DPG_ASAN) >= max(os.path.getmtime(d) for d in deps)):
        os.makedirs(DPG_ASAN_DIR, exist_ok=True)
        obj = os.path.join(DPG_ASAN_DIR, "dpg_host.o")
        # host-only sanitizer build: -fno-gpu-sanitize keeps any device pass
        # unsanitized (the pool runs no GPU sanitizer builds)
        san = ["-fsanitize=address,undefined", "-fno-gpu-sanitize", "-fno-sanitize-recover=undefined"]
        subprocess.run([HIPCC, "--cuda-host-only", "-O1", "-g", "-std=c++17", "-fPIC", "-c"] + san +
                       ["-fno-omit-frame-pointer", "-o", obj, os.path.join(src, "dpg_api.hip")],
                       check=True, cwd=DPG_ASAN_DIR)
        # no device code: the fat binary the host object registers at load
        # is an empty stand-in (nothing here launches a kernel)
        und = subprocess.run(["nm", "-u", obj], check=True, capture_output=True, text=True).stdout
        syms = sorted(set(re.findall(r"__hip_fatbin_[0-9a-f]+", und)))
        stub = os.path.join(DPG_ASAN_DIR, "fatbin_stub.c")
        with open(stub, "w") as fh:
            for sym in syms:
                fh.write(f"char {sym}[64] __attribute__((aligned(4096))) = {{0}};\n")
        subprocess.run(["/opt/rocm/lib/llvm/bin/clang", "-c", "-fPIC", "-o", stub + ".o", stub],
                       check=True)
        tmp = DPG_ASAN + f".{os.getpid()}.tmp"
        subprocess.run([HIPCC, "-shared", "-fsanitize=address,undefined", "-fno-gpu-sanitize", "-o", tmp,
                        obj, stub + ".o"], check=True, cwd=DPG_ASAN_DIR)
        os.replace(tmp, DPG_ASAN)
    return DPG_ASAN


def test_oracle_tests_under_asan(oracle_asan):
    files = ["tests/test_oracle_golden.py", "tests/test_sampling_distribution.py",
             "tests/test_mechanisms.py"]
    probe = ("import oracle.oracle as o; import sys; "
             "sys.exit(0 if o._LIB.endswith('asan/libdporacle.so') else 3)")
    r = subprocess.run([sys.executable, "-c", probe], env=_env(DPO_LIB_PATH=oracle_asan),
                       cwd=ROOT, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        "-m", "not gpu"] + files,
                       env=_env(DPO_LIB_PATH=oracle_asan), cwd=ROOT, capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert "passed" in r.stdout


# Every entry point on its argument-error path (a null context or null
# buffers), the pure helpers, and the context constructor without a device.
_DRIVER = r"""
import ctypes, sys
L = ctypes.CDLL(sys.argv[1])
vp, i64, i32, u64 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_uint64
INVALID = -1
L.dpg_stream_seed.restype = u64
L.dpg_stream_seed.argtypes = [u64, u64]
a, b = L.dpg_stream_seed(1, 2), L.dpg_stream_seed(1, 3)
assert a != b and a == L.dpg_stream_seed(1, 2)
buf = ctypes.create_string_buffer(64)
L.dpg_last_error.argtypes = [vp, ctypes.c_char_p, ctypes.c_size_t]
L.dpg_last_error(None, buf, 64)
L.dpg_last_error(None, None, 0)
L.dpg_ctx_destroy.argtypes = [vp]
L.dpg_ctx_destroy(None)
rc = {}
rc["set_seed"] = L.dpg_set_seed(vp(), u64(7))
rc["set_tuning"] = L.dpg_set_tuning(vp(), i32(256), i32(512))
rc["bound_aggregate"] = L.dpg_bound_aggregate(vp(), vp(), vp(), vp(), i64(10), vp(), vp(), vp())
rc["select_and_noise"] = L.dpg_select_and_noise(vp(), vp(), vp(), vp(), vp(), vp(), vp())
rc["compact_kept"] = L.dpg_compact_kept(vp(), vp(), vp(), i64(10), i32(1), vp(), vp(), vp(), vp())
rc["preaggregate"] = L.dpg_preaggregate(vp(), vp(), vp(), vp(), i64(10), vp(), vp(), i64(0), vp(), vp(), vp())
rc["utility_analysis"] = L.dpg_utility_analysis(vp(), vp(), vp(), i64(0), vp(), vp(), vp(), vp(), vp(), vp(), vp())
rc["dataset_histograms"] = L.dpg_dataset_histograms(vp(), vp(), i64(0), vp(), i64(0), i32(0), vp(), vp())
rc["ctx_create_comm"] = L.dpg_ctx_create_comm(vp(), vp(), i32(0), i32(1))
rc["reduce_scatter_partials"] = L.dpg_reduce_scatter_partials(vp(), vp(), vp(), vp(), vp(), vp())
rc["last_stage_times"] = L.dpg_last_stage_times(vp(), vp(), ctypes.c_size_t(0), vp(), i32(0), vp())
bad = {k: v for k, v in rc.items() if v == 0}
assert not bad, f"accepted a null context: {bad}"
L.dpg_comm_unique_id.argtypes = [vp]
L.dpg_comm_unique_id(None)
L.dpg_ctx_create.restype = vp
L.dpg_ctx_create.argtypes = [ctypes.c_int, u64]
ctx = L.dpg_ctx_create(0, 1)  # no device here: expected null, must not crash
if ctx:
    L.dpg_ctx_destroy(ctx)
print("ok", len(rc))
"""


def test_c_abi_host_paths_under_asan(dpg_asan):
    r = subprocess.run([sys.executable, "-c", _DRIVER, dpg_asan], env=_env(HIP_VISIBLE_DEVICES=""),
                       cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert r.stdout.startswith("ok"), r.stdout

"""The C-ABI library loads, exports every symbol include/dpg.h declares, and
the ctypes struct layouts match the C compiler's (no GPU needed)."""
import ctypes
import os
import re
import subprocess
import tempfile

import pytest

from pipelinedp_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dpg.h")


def declared_functions():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(dpg_\w+)\s*\(", text)))


def test_header_and_binding_agree():
    assert sorted(_native.EXPORTED) == declared_functions()


def test_library_exports_every_symbol(built):
    lib = ctypes.CDLL(_native.library_path())
    for name in declared_functions():
        assert hasattr(lib, name), name
    _native.load()


def test_struct_layouts_match_c(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "dpg.h"\n'
                   'int main(){printf("%zu %zu %zu %zu %zu %zu %zu %zu\\n",'
                   'sizeof(dpg_bound_params), sizeof(dpg_partials), sizeof(dpg_select_params),'
                   'sizeof(dpg_noise_params), offsetof(dpg_bound_params, public_mask),'
                   'offsetof(dpg_select_params, public_mask), offsetof(dpg_noise_params, msq_const_value),'
                   'offsetof(dpg_bound_params, rec_id_offset));'
                   'printf("%zu %zu %zu %zu %zu\\n", sizeof(dpg_pair_entry), sizeof(dpg_ua_config),'
                   'sizeof(dpg_ua_params), offsetof(dpg_ua_config, keep_table),'
                   'offsetof(dpg_ua_params, public_mask));}')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    want = [ctypes.sizeof(_native.BoundParams), ctypes.sizeof(_native.Partials),
            ctypes.sizeof(_native.SelectParams), ctypes.sizeof(_native.NoiseParams),
            _native.BoundParams.public_mask.offset, _native.SelectParams.public_mask.offset,
            _native.NoiseParams.msq_const_value.offset, _native.BoundParams.rec_id_offset.offset,
            ctypes.sizeof(_native.PairEntry), ctypes.sizeof(_native.UaConfig),
            ctypes.sizeof(_native.UaParams), _native.UaConfig.keep_table.offset,
            _native.UaParams.public_mask.offset]
    assert got == want


def test_stream_seed_matches_oracle(built):
    """dpg_stream_seed (pure host function) equals the oracle's restatement,
    and distinct nonces give distinct stream seeds."""
    from oracle import oracle
    seeds = set()
    for seed in (0, 1, 0x5EED, 2**64 - 1):
        for nonce in (0, 1, 2, 0xDEADBEEF, 2**63):
            s = _native.stream_seed(seed, nonce)
            assert s == oracle.stream_seed(seed, nonce)
            seeds.add(s)
    assert len(seeds) == 20


def test_no_cpu_fallback_without_gpu():
    import torch
    import pipelinedp_amd as pdp
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    backend = pdp.MI355XBackend(device=0, seed=1)
    with pytest.raises(_native.NativeError, match="no CPU fallback"):
        backend.ctx

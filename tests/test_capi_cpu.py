"""CPU-only checks of the C ABI: the library loads, exports every symbol the header
declares, and the ctypes prototypes/structures match the header.  No compute calls."""
import ctypes as C
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "ngrtd.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ngrtd_[a-z_0-9]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    import __graft_entry__ as g
    g.build()
    from noblegas_rtd_mcmc_amd import _lib
    return _lib.load()


def test_every_declared_symbol_is_exported_and_bound(lib):
    from noblegas_rtd_mcmc_amd import _lib
    names = header_functions()
    assert len(names) >= 19
    for n in names:
        assert hasattr(lib, n), n
        assert n in _lib.PROTOTYPES, n
    assert set(_lib.PROTOTYPES) == set(names)
    assert lib.ngrtd_abi_version() == 1


def test_exports_are_c_abi(lib):
    from noblegas_rtd_mcmc_amd import _lib
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (ngrtd_\w+)", out))
    assert set(header_functions()) <= exported


def test_struct_layout_matches_header():
    """Compile a tiny C program that prints sizeof/offsetof of the descriptor structs and
    compare with ctypes."""
    from noblegas_rtd_mcmc_amd import _lib
    src = r'''
#include <stdio.h>
#include <stddef.h>
#include "ngrtd.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu\n", sizeof(ngrtd_model_desc), sizeof(ngrtd_tracer_desc),
         offsetof(ngrtd_model_desc, tracers), offsetof(ngrtd_model_desc, rtd_obs),
         offsetof(ngrtd_model_desc, rtd_nu_b), offsetof(ngrtd_model_desc, ce_beta_b));
  printf("%zu %zu %zu %zu %zu %zu\n", sizeof(ngrtd_demcz_state), offsetof(ngrtd_demcz_state, hist_cap),
         offsetof(ngrtd_demcz_state, tune_interval), offsetof(ngrtd_demcz_state, drop_fraction),
         offsetof(ngrtd_demcz_state, seed), offsetof(ngrtd_demcz_state, tr_b));
  return 0;
}'''
    tmp = "/tmp/ngrtd_layout_%d" % os.getpid()
    with open(tmp + ".c", "w") as f:
        f.write(src)
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), tmp + ".c", "-o", tmp], check=True)
    vals = [int(x) for x in subprocess.run([tmp], capture_output=True, text=True).stdout.split()]
    M, T, Z = _lib.ModelDesc, _lib.TracerDesc, _lib.DemczState
    assert vals == [C.sizeof(M), C.sizeof(T), M.tracers.offset, M.rtd_obs.offset, M.rtd_nu_b.offset,
                    M.ce_beta_b.offset, C.sizeof(Z), Z.hist_cap.offset, Z.tune_interval.offset,
                    Z.drop_fraction.offset, Z.seed.offset, Z.tr_b.offset]


def test_roles_match_spec():
    from noblegas_rtd_mcmc_amd import spec, engine
    assert tuple(spec.ROLES) == tuple(engine.ROLE_ORDER)
    src = open(HEADER).read()
    for i, r in enumerate(spec.ROLES):
        name = {"Ae_beta": "AE_BETA", "F_beta": "F_BETA", "E_beta": "E_BETA", "m": "M", "b_beta": "B_BETA",
                "nu_ce_beta": "NU_CE_BETA", "thalf_cfc_beta": "THALF_BETA", "nu_rtd_beta": "NU_RTD_BETA"}.get(r, r.upper())
        assert re.search(r"NGRTD_ROLE_%s\s*=\s*%d\b" % (name, i), src), r


def test_no_gpu_means_loud_failure():
    """Without a visible GPU the engine refuses to run (no silent CPU fallback)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from noblegas_rtd_mcmc_amd import _lib
    with pytest.raises(_lib.NgrtdError):
        _lib.Context(0)

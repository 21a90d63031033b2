"""CPU checks of the drop-in boundary: the C-ABI library loads and exports every entry point
that include/rcmdyn.h declares, the ctypes image of rcmdyn_config matches the C layout, and
the host-only decomposition entry points agree with mpplib's rule.  No compute call is made."""
import ctypes
import os
import re
import subprocess
import tempfile

import pytest

from regcm_amd import dycore
from regcm_amd.config import RcmdynConfig, set_nproc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rcmdyn.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(rcmdyn_\w+)\s*\(", src, re.M)))


def test_header_declarations_exported():
    names = declared_functions()
    assert len(names) >= 15
    L = dycore.lib()
    for n in names:
        assert hasattr(L, n), n
    assert sorted(dycore.EXPORTED) == names


def test_exported_symbols_in_elf():
    out = subprocess.run(["nm", "-D", "--defined-only", dycore.LIB_PATH], capture_output=True, text=True).stdout
    for n in declared_functions():
        assert re.search(rf"\bT {n}$", out, re.M), n


def test_config_layout_matches_c():
    probe = r"""
#include <stdio.h>
#include <stddef.h>
#include "rcmdyn.h"
#define O(f) printf("%s %zu\n", #f, offsetof(rcmdyn_config, f))
int main(void) {
  printf("size %zu\n", sizeof(rcmdyn_config));
  O(jx); O(present_qc); O(ds); O(dtbdys); O(sigma); O(zmatx); O(zmatxr); O(am); O(tau);
  O(varpa1); O(an); O(hbar); O(aam); O(dtau); O(sigmah); O(pd); O(comm_rank); O(device);
  O(comm_unique_id); O(nh_dtsmax); O(rhmin); O(rhmax); O(isladvec); O(iqmsl); O(ibltyp); O(nuk);
  O(tkemin); O(ipptls); O(nqx); O(i_band); O(i_crm); O(ichem);
  return 0;
}
"""
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "p.c")
        open(c, "w").write(probe)
        exe = os.path.join(d, "p")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), "-o", exe, c], check=True)
        lines = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split("\n")
    got = dict(l.split() for l in lines if l)
    assert int(got.pop("size")) == ctypes.sizeof(RcmdynConfig)
    for name, off in got.items():
        assert getattr(RcmdynConfig, name).offset == int(off), name


@pytest.mark.parametrize("n", [1, 2, 3, 4, 6, 8, 12, 16])
@pytest.mark.parametrize("shape", [(192, 192), (384, 192), (96, 200), (48, 48)])
def test_set_nproc_c_matches_python(n, shape):
    assert dycore.set_nproc(n, *shape) == set_nproc(n, *shape)


def test_tile_extents_partition_domain():
    """Tiles cover the dot grid exactly once; remainder points go to the low tiles and the
    last tile in each direction has one fewer cross point (mod_mppparam.F90:1295-1360)."""
    jx, iy = 97, 50
    cj, ci = 3, 2
    cover = [[0] * (jx + 1) for _ in range(iy + 1)]
    for t in range(cj * ci):
        ext, bdy = dycore.tile_extent(jx, iy, cj, ci, t)
        jde1, jde2, ide1, ide2, jce1, jce2, ice1, ice2 = ext
        for i in range(ide1, ide2 + 1):
            for j in range(jde1, jde2 + 1):
                cover[i][j] += 1
        assert jce2 == (jde2 - 1 if jde2 == jx else jde2)
        assert ice2 == (ide2 - 1 if ide2 == iy else ide2)
        assert bdy == [t // ci == 0, t // ci == cj - 1, t % ci == 0, t % ci == ci - 1]
    assert all(cover[i][j] == 1 for i in range(1, iy + 1) for j in range(1, jx + 1))
    widths = [dycore.tile_extent(jx, iy, cj, ci, t * ci)[0][1] - dycore.tile_extent(jx, iy, cj, ci, t * ci)[0][0] + 1
              for t in range(cj)]
    assert widths == [33, 32, 32]


@pytest.mark.parametrize("band,crm", [(1, 0), (1, 1)])
def test_tile_extents_periodic(band, crm):
    """rcmdyn_tile_extent_cfg: a periodic direction (i_band: j, i_crm: i) has no boundary side
    on any tile and its cross range takes every point (mod_mppparam.F90:1131-1132, 1340-1360);
    the tiles still cover the dot grid exactly once, and the other direction is unchanged.  CRM
    without the band is refused, as rcmdyn_create refuses it."""
    jx, iy = 97, 50
    cj, ci = 3, 2
    with pytest.raises(dycore.EngineError):
        dycore.tile_extent(jx, iy, cj, ci, 0, i_band=0, i_crm=1)
    cover = [[0] * (jx + 1) for _ in range(iy + 1)]
    for t in range(cj * ci):
        ext, bdy = dycore.tile_extent(jx, iy, cj, ci, t, i_band=band, i_crm=crm)
        plain, pbdy = dycore.tile_extent(jx, iy, cj, ci, t)
        jde1, jde2, ide1, ide2, jce1, jce2, ice1, ice2 = ext
        assert ext[:4] == plain[:4]
        for i in range(ide1, ide2 + 1):
            for j in range(jde1, jde2 + 1):
                cover[i][j] += 1
        assert jce2 == (jde2 if band else plain[5])
        assert ice2 == (ide2 if crm else plain[7])
        assert bdy[:2] == ([0, 0] if band else pbdy[:2])
        assert bdy[2:] == ([0, 0] if crm else pbdy[2:])
    assert all(cover[i][j] == 1 for i in range(1, iy + 1) for j in range(1, jx + 1))


@pytest.mark.parametrize("bad,msg", [(dict(i_band=0), "i_crm"), (dict(idynamic=1), "i_crm"),
                                     (dict(i_crm=0), "iboudy = 0"), (dict(idiffu=3), "idiffu = 3")],
                         ids=["crm-without-band", "crm-hydrostatic", "iboudy0-lam", "nh-band-idiffu3"])
def test_periodic_refusals(bad, msg):
    """CRM is built for the non-hydrostatic core over the band (PreProc/CRM/crm_test.in);
    iboudy = 0 only where no boundary line exists (CRM); the sixth-order diffusion not on the
    NH band.  Refused at create, before any device is touched."""
    import dataclasses
    from regcm_amd.config import CONFIGS
    from regcm_amd import icbc
    rc = dataclasses.replace(CONFIGS["CRM"], **bad)
    data = icbc.generate_crm(CONFIGS["CRM"])
    with pytest.raises(dycore.EngineError, match=msg):
        dycore.DynCore(rc, data["split"])


def test_create_without_gpu_fails_loudly():
    """On a host without a GPU the engine refuses to start (no silent CPU fallback)."""
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    from regcm_amd.config import CONFIGS
    from regcm_amd import icbc
    rc = CONFIGS["C1"]
    data = icbc.generate(rc)
    with pytest.raises(dycore.EngineError):
        dycore.DynCore(rc, data["split"])


@pytest.mark.parametrize("opt,msg", [({"upstream_mode": 2}, "upstream_mode"),
                                     ({"idiffu": 4}, "idiffu"), ({"idiffu": 0}, "idiffu"),
                                     ({"iboudy": 0}, "iboudy"),
                                     ({"ibltyp": 2, "iuwvadv": 2}, "iuwvadv"),
                                     ({"ipptls": 0}, "ipptls"), ({"ipptls": 3}, "ipptls"),
                                     ({"i_band": 2}, "i_band"), ({"i_crm": 1}, "i_crm"),
                                     ({"ichem": 1}, "ichem")])
def test_create_refuses_unbuilt_options(opt, msg):
    """A drop-in refuses what it does not compute: option values whose reference branches are
    not built fail rcmdyn_create with the option's name, before any device call (so here too)."""
    import dataclasses
    from regcm_amd.config import CONFIGS
    from regcm_amd import icbc
    rc = dataclasses.replace(CONFIGS["C1"], **opt)
    data = icbc.generate(CONFIGS["C1"])
    with pytest.raises(dycore.EngineError, match=msg):
        dycore.DynCore(rc, data["split"])


@pytest.mark.parametrize("mode", ["init", "split", "two"])
def test_create_refuses_removed_rccl_channel_modes(monkeypatch, mode):
    """RCMDYN_RCCL_CHAN2 has one mode left ("one": both streams share the job's communicator);
    the removed second-communicator modes and any other value fail rcmdyn_create."""
    from regcm_amd.config import CONFIGS
    from regcm_amd import icbc
    monkeypatch.setenv("RCMDYN_RCCL_CHAN2", mode)
    rc = CONFIGS["C1"]
    data = icbc.generate(rc)
    with pytest.raises(dycore.EngineError, match="RCMDYN_RCCL_CHAN2"):
        dycore.DynCore(rc, data["split"])


def test_field_enum_matches_header_python_fortran():
    """rcmdyn_field order is one contract for C, the Python host and the Fortran shim."""
    from regcm_amd.config import FIELD_NAMES
    src = open(HEADER).read()
    body = src[src.index("enum rcmdyn_field"):src.index("RCMDYN_NFIELDS")]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    names = re.findall(r"RCMDYN_(\w+)", body)
    assert names == FIELD_NAMES
    f90 = open(os.path.join(ROOT, "regcm_amd", "fortran", "mod_gpu_dyn.F90")).read()
    ids = {m.group(1).upper(): int(m.group(2)) for m in re.finditer(r"\bf_(\w+)\s*=\s*(\d+)", f90)}
    assert ids == {n: q for q, n in enumerate(FIELD_NAMES)}


@pytest.mark.parametrize("ipptls,nqx", [(1, 5), (2, 2), (1, 3), (2, 4)])
def test_create_refuses_nqx_not_matching_ipptls(ipptls, nqx):
    """nqx is what param derives from ipptls (Main/mod_params.F90:1358-1366): 2 for ipptls = 1,
    5 for ipptls = 2; any other pairing is refused before a device call."""
    import ctypes
    import dataclasses
    from regcm_amd.config import CONFIGS, build_config
    from regcm_amd import icbc
    rc = dataclasses.replace(CONFIGS["C1"], ipptls=ipptls)
    data = icbc.generate(CONFIGS["C1"])
    cfg = build_config(rc, data["split"])
    cfg.nqx = nqx
    h = ctypes.c_void_p()
    assert dycore.lib().rcmdyn_create(ctypes.byref(cfg), ctypes.byref(h)) != 0
    assert b"nqx" in dycore.lib().rcmdyn_last_error(None)


def test_exchange_plan_carries_the_hydrometeors():
    """nqx = 5: the prologue messages grow by qi, qr, qs (atm1 2 wide, atm2 3 wide), and every
    rank's sends still match its neighbours' receives."""
    import dataclasses
    import numpy as np
    from regcm_amd.config import CONFIGS
    from regcm_amd import icbc
    rc = CONFIGS["C1"]
    data = icbc.generate(rc)
    p2 = dycore.exchange_plan(rc, data["split"], 2, 2, 0, 2)
    p5 = dycore.exchange_plan(dataclasses.replace(rc, ipptls=2), data["split"], 2, 2, 0, 2)
    assert p5[:, 5].sum() > p2[:, 5].sum()
    plans = [dycore.exchange_plan(dataclasses.replace(rc, ipptls=2), data["split"], 2, 2, r, 2) for r in range(4)]
    for a in range(4):
        for b in range(4):
            sa = [tuple(x[[2, 5, 6]]) for x in plans[a] if x[1] == 1 and x[3] == 0 and x[4] == b]
            rb = [tuple(x[[2, 5, 6]]) for x in plans[b] if x[1] == 1 and x[3] == 1 and x[4] == a]
            assert sa == rb, (a, b)
    assert np.all(p5[:, 1] > 0)


def test_bench_loads_engine_before_torch():
    """bench.py binds the engine (and /opt/rocm's librccl.so.1) before torch can load its own
    copy under the same soname, on every rank, and reports each rank's runtime."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    body = src[src.index("def main():"):]
    assert "import torch" not in src[:src.index("def main():")]
    assert body.index("rt = runtime_info()") < body.index("import torch")
    assert "runtime_per_rank" in body


def test_overlap_shares_on_the_scaling_tiles():
    """rcmdyn_overlap_shares (host-only): on C3's 2/4/8-GPU tiles part 1 of k_momentum and
    k_scalars (the blocks beside the prologue exchange) is non-empty -- the block columns are
    shifted so one lies inside R -- and k_columns' part 1 is R itself."""
    from regcm_amd.config import CONFIGS, set_nproc
    from regcm_amd import icbc
    rc = CONFIGS["C3"]
    data = icbc.generate(rc)
    for n, lo in ((2, 0.6), (4, 0.5), (8, 0.4)):
        cj, ci = set_nproc(n, rc.jx, rc.iy)
        sh = dycore.overlap_shares(rc, data["split"], cj, ci)
        assert len(sh) == n
        tot = [sum(x[q] for x in sh) for q in range(6)]
        assert tot[0] / tot[1] > 0.9
        assert tot[2] / tot[3] > lo and tot[4] / tot[5] > lo, (n, tot)
    one = dycore.overlap_shares(rc, data["split"], 1, 1)
    assert one[0][0] == 0 and one[0][2] == 0 and one[0][4] == 0

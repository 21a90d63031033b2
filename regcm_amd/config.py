"""Run configuration for the dynamical-core engine.

Mirrors the namelist groups / run-time globals the reference dyn core reads:
``Share/mod_dynparam.F90:453-476`` (dimparam, boundaryparam), ``Main/mod_params.F90:85-170``
(physicsparam, dynparam, hydroparam) with the defaults of ``Main/mod_params.F90:194-300`` and
the hydrostatic dynparam overrides of ``Main/mod_params.F90:645-661``.

``RcmdynConfig`` is the ctypes image of ``rcmdyn_config`` in ``include/rcmdyn.h``.
"""
from __future__ import annotations

import ctypes
import dataclasses
from typing import Optional, Sequence

import numpy as np

MAXKZ = 64
MAXSPLIT = 4
ABI_VERSION = 6

# Share/mod_sigma.F90:88-152 -- the hard-coded sigma tables (data, cited).
SIGMA_TABLES = {
    14: [0.0, 0.04, 0.10, 0.17, 0.25, 0.35, 0.46, 0.56, 0.67, 0.77, 0.86, 0.93, 0.97,
         0.99, 1.0],
    18: [0.0, 0.05, 0.10, 0.16, 0.23, 0.31, 0.39, 0.47, 0.55, 0.63, 0.71, 0.78, 0.84,
         0.89, 0.93, 0.96, 0.98, 0.99, 1.0],
    23: [0.0, 0.05, 0.1, 0.15, 0.2, 0.25, 0.3, 0.35, 0.4, 0.45, 0.5, 0.55, 0.6, 0.65,
         0.7, 0.75, 0.8, 0.85, 0.89, 0.93, 0.96, 0.98, 0.99, 1.0],
    41: [0.0000, 0.0500, 0.0978, 0.1436, 0.1875, 0.2295, 0.2697, 0.3082, 0.3451, 0.3804,
         0.4143, 0.4468, 0.4779, 0.5078, 0.5364, 0.5639, 0.5903, 0.6156, 0.6399, 0.6632,
         0.6856, 0.7071, 0.7277, 0.7476, 0.7667, 0.7850, 0.8027, 0.8196, 0.8359, 0.8516,
         0.8667, 0.8812, 0.8952, 0.9087, 0.9216, 0.9341, 0.9461, 0.9577, 0.9689, 0.9796,
         0.9900, 1.0000],
}


class RcmdynConfig(ctypes.Structure):
    """ctypes image of ``rcmdyn_config`` (include/rcmdyn.h)."""

    _fields_ = [
        ("abi_version", ctypes.c_int32),
        ("jx", ctypes.c_int32), ("iy", ctypes.c_int32), ("kz", ctypes.c_int32),
        ("nproc_j", ctypes.c_int32), ("nproc_i", ctypes.c_int32),
        ("tile_first", ctypes.c_int32), ("tile_count", ctypes.c_int32),
        ("idynamic", ctypes.c_int32), ("iboudy", ctypes.c_int32),
        ("idiffu", ctypes.c_int32), ("ipgf", ctypes.c_int32), ("nsplit", ctypes.c_int32),
        ("nspgx", ctypes.c_int32), ("nspgd", ctypes.c_int32),
        ("diffu_hgtf", ctypes.c_int32), ("upstream_mode", ctypes.c_int32),
        ("stability_enhance", ctypes.c_int32), ("present_qc", ctypes.c_int32),
        ("ds", ctypes.c_double), ("dtsec", ctypes.c_double), ("ptop", ctypes.c_double),
        ("gnu1", ctypes.c_double), ("gnu2", ctypes.c_double), ("uoffc", ctypes.c_double),
        ("t_extrema", ctypes.c_double), ("q_rel_extrema", ctypes.c_double),
        ("ckh", ctypes.c_double), ("adyndif", ctypes.c_double),
        ("high_nudge", ctypes.c_double), ("medium_nudge", ctypes.c_double),
        ("low_nudge", ctypes.c_double), ("bdy_nm", ctypes.c_double),
        ("bdy_dm", ctypes.c_double), ("dtbdys", ctypes.c_double),
        ("sigma", ctypes.c_double * (MAXKZ + 1)),
        ("zmatx", (ctypes.c_double * MAXKZ) * MAXSPLIT),
        ("zmatxr", (ctypes.c_double * MAXKZ) * MAXSPLIT),
        ("am", (ctypes.c_double * MAXKZ) * MAXSPLIT),
        ("tau", (ctypes.c_double * MAXKZ) * MAXSPLIT),
        ("varpa1", (ctypes.c_double * (MAXKZ + 1)) * MAXSPLIT),
        ("an", ctypes.c_double * MAXSPLIT), ("hbar", ctypes.c_double * MAXSPLIT),
        ("aam", ctypes.c_double * MAXSPLIT), ("dtau", ctypes.c_double * MAXSPLIT),
        ("sigmah", ctypes.c_double * (MAXKZ + 1)), ("pd", ctypes.c_double),
        ("comm_rank", ctypes.c_int32), ("comm_size", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("comm_unique_id", ctypes.c_uint8 * 128),
        ("ifupr", ctypes.c_int32), ("ifrayd", ctypes.c_int32), ("rayndamp", ctypes.c_int32),
        ("nh_reserved", ctypes.c_int32),
        ("nhbet", ctypes.c_double), ("nhxkd", ctypes.c_double),
        ("rayalpha0", ctypes.c_double), ("rayhd", ctypes.c_double),
        ("nh_dtsmax", ctypes.c_double), ("nh_xmsf", ctypes.c_double),
        ("rhmin", ctypes.c_double), ("rhmax", ctypes.c_double),
        ("isladvec", ctypes.c_int32), ("iqmsl", ctypes.c_int32),
        ("ibltyp", ctypes.c_int32), ("iuwvadv", ctypes.c_int32),
        ("nuk", ctypes.c_double), ("tkemin", ctypes.c_double),
        ("ipptls", ctypes.c_int32), ("nqx", ctypes.c_int32),
        ("i_band", ctypes.c_int32), ("i_crm", ctypes.c_int32), ("ichem", ctypes.c_int32),
    ]


# Field ids, enum rcmdyn_field in include/rcmdyn.h (same order).
FIELD_NAMES = [
    "ATM1_U", "ATM1_V", "ATM1_T", "ATM1_QV", "ATM1_QC",
    "ATM2_U", "ATM2_V", "ATM2_T", "ATM2_QV", "ATM2_QC",
    "PSA", "PSB", "DSTOR", "HSTOR",
    "MSFX", "MSFD", "CORIOL", "HT",
    "XUB_B0", "XUB_BT", "XVB_B0", "XVB_BT", "XTB_B0", "XTB_BT", "XQB_B0", "XQB_BT",
    "XPSB_B0", "XPSB_BT",
    "PSC", "PTEN", "PSDOTA", "TTEN", "UTEN", "VTEN", "QVTEN", "QCTEN",
    "OMEGA", "QDOT", "XKC", "PHI",
    "ATM1_PP", "ATM2_PP", "ATM1_W", "ATM2_W", "XPPB_B0", "XPPB_BT", "XWWB_B0", "XWWB_BT",
    "ATM0_PS", "ATM0_PR", "ATM0_T", "ATM0_RHO", "ATM0_Z", "ATM0_PF", "ATM0_RHOF", "ATM0_ZF",
    "DPSDXM", "DPSDYM", "DPRDDX", "DPRDDY", "EF", "DDX", "DDY", "DMDX", "DMDY", "EX", "CRX", "CRY",
    "TPHY", "QVPHY", "QCPHY", "UPHY", "VPHY", "PPPHY", "WPHY",
    "ATMS_UBX3D", "ATMS_VBX3D", "ATMS_UBD3D", "ATMS_VBD3D", "ATMS_TB3D", "ATMS_QVB3D", "ATMS_QCB3D",
    "ATMS_TV3D", "ATMS_PB3D", "ATMS_PF3D", "ATMS_PS2D", "ATMS_RHOX2D", "ATMS_TH3D", "ATMS_RHOB3D",
    "ATMS_TP3D", "ATMS_WPX3D", "ATMS_WB3D", "ATMS_ZQ", "ATMS_ZA", "ATMS_DZQ", "ATMS_QSB3D", "ATMS_RHB3D",
    "XUB_B1", "XVB_B1", "XTB_B1", "XQB_B1", "XPSB_B1", "XPPB_B1", "XWWB_B1", "ATM0_PSDOT",
    "ATM1_TKE", "ATM2_TKE", "TKEPHY", "KPBL",
    "ATM1_QI", "ATM1_QR", "ATM1_QS", "ATM2_QI", "ATM2_QR", "ATM2_QS",
    "QIPHY", "QRPHY", "QSPHY", "ATMS_QXB3D_QI", "ATMS_QXB3D_QR", "ATMS_QXB3D_QS",
]
FIELD = {n: i for i, n in enumerate(FIELD_NAMES)}
TWO_D = {"PSA", "PSB", "MSFX", "MSFD", "CORIOL", "HT", "XPSB_B0", "XPSB_BT", "PSC",
         "PTEN", "PSDOTA", "ATM0_PS", "DPSDXM", "DPSDYM", "EF", "DDX", "DDY", "DMDX", "DMDY",
         "EX", "CRX", "CRY", "ATMS_PS2D", "ATMS_RHOX2D", "XPSB_B1", "ATM0_PSDOT", "KPBL"}
FULL_LEVELS = {"QDOT", "ATM1_W", "ATM2_W", "XWWB_B0", "XWWB_BT", "ATM0_PF", "ATM0_RHOF",
               "ATM0_ZF", "WPHY", "ATMS_PF3D", "ATMS_WB3D", "ATMS_ZQ", "XWWB_B1",
               "ATM1_TKE", "ATM2_TKE", "TKEPHY"}
TKE_STATE_FIELDS = ["ATM1_TKE", "ATM2_TKE"]
# nqx = 5 (ipptls >= 2): the ice, rain and snow hydrometeors and their physics / slice fields
QX_STATE_FIELDS = ["ATM1_QI", "ATM1_QR", "ATM1_QS", "ATM2_QI", "ATM2_QR", "ATM2_QS"]
QX_PHY_FIELDS = ["QIPHY", "QRPHY", "QSPHY"]
# physics coupling seam: pc_physic tendencies (put) and the mkslice export (get)
PHY_FIELDS = ["TPHY", "QVPHY", "QCPHY", "UPHY", "VPHY"]
NH_PHY_FIELDS = ["PPPHY", "WPHY"]
ATMS_FIELDS = [n for n in FIELD_NAMES if n.startswith("ATMS_") and not n.startswith("ATMS_QXB3D")]
QX_ATMS_FIELDS = ["ATMS_QXB3D_QI", "ATMS_QXB3D_QR", "ATMS_QXB3D_QS"]
NH_STATE_FIELDS = ["ATM1_PP", "ATM2_PP", "ATM1_W", "ATM2_W"]
NH_BDY_FIELDS = ["XPPB_B0", "XPPB_BT", "XWWB_B0", "XWWB_BT"]
NH_STATIC_FIELDS = ["ATM0_PS", "ATM0_PR", "ATM0_T", "ATM0_RHO", "ATM0_Z", "ATM0_PF",
                    "ATM0_RHOF", "ATM0_ZF", "DPSDXM", "DPSDYM", "DPRDDX", "DPRDDY",
                    "EF", "DDX", "DDY", "DMDX", "DMDY", "EX", "CRX", "CRY"]
STATE_FIELDS = ["ATM1_U", "ATM1_V", "ATM1_T", "ATM1_QV", "ATM1_QC",
                "ATM2_U", "ATM2_V", "ATM2_T", "ATM2_QV", "ATM2_QC",
                "PSA", "PSB", "DSTOR", "HSTOR"]
STATIC_FIELDS = ["MSFX", "MSFD", "CORIOL", "HT"]
BDY_FIELDS = ["XUB_B0", "XUB_BT", "XVB_B0", "XVB_BT", "XTB_B0", "XTB_BT",
              "XQB_B0", "XQB_BT", "XPSB_B0", "XPSB_BT"]


def field_levels(name: str, kz: int, nsplit: int) -> int:
    if name in TWO_D:
        return 1
    if name in ("DSTOR", "HSTOR"):
        return nsplit
    if name in FULL_LEVELS:
        return kz + 1
    return kz


@dataclasses.dataclass
class RunConfig:
    """One BASELINE.json configuration (physics stubbed).  ``idynamic`` 1 = hydrostatic,
    2 = non-hydrostatic; the NH knobs are nonhydroparam (Main/mod_params.F90:287-296) and
    referenceatm (Share/mod_dynparam.F90:507-508)."""

    jx: int
    iy: int
    kz: int
    ds: float            # km
    dt: float            # s (namelist dt == dtsec)
    ptop: float = 5.0    # cb
    iboudy: int = 5
    idiffu: int = 1
    ipgf: int = 0
    nsplit: int = 2
    nspgx: Optional[int] = None
    nspgd: Optional[int] = None
    diffu_hgtf: int = 1
    upstream_mode: int = 1           # dynparam; 0 = .false. (centred advection)
    gnu1: float = 0.0625
    gnu2: float = 0.0625
    uoffc: float = 0.25
    t_extrema: float = 5.0
    q_rel_extrema: float = 0.20
    ckh: float = 1.0
    adyndif: float = 1.0
    high_nudge: float = 3.0
    medium_nudge: float = 2.0
    low_nudge: float = 1.0
    bdy_nm: float = -1.0
    bdy_dm: float = -1.0
    ibdyfrq: int = 6
    present_qc: int = 0
    stability_enhance: int = 1       # dynparam (Main/mod_params.F90:646); 0 drops the extrema limiters
    name: str = ""
    idynamic: int = 1
    ifupr: int = 1
    ifrayd: int = 1
    rayndamp: int = 5
    rayalpha0: float = 0.0003
    rayhd: float = 10000.0
    rhmin: float = 0.01              # cldparam, Main/mod_params.F90:331-332
    rhmax: float = 1.01
    isladvec: int = 0                # physicsparam, Main/mod_params.F90:243-244
    iqmsl: int = 1
    ibltyp: int = 1                  # physicsparam; 2 = UW PBL (TKE advected by the dyn step)
    nuk: float = 5.0                 # uwparam, Main/mod_params.F90:480
    iuwvadv: int = 0                 # uwparam; 1 with ibltyp = 2: PBL-aware qc vertical flux (vadv4d ind = 3)
    ipptls: int = 1                  # physicsparam; > 1 (WSM5 / NT): nqx = 5, Main/mod_params.F90:1358-1366
    i_band: int = 0                  # 1: tropical band, periodic in j (hydrostatic core only)
    # i_crm, ichem: physicsparam options the engine refuses
    i_crm: int = 0
    ichem: int = 0
    tkemin: float = 1.0e-3           # uwtkemin, Main/pbllib/mod_pbl_uwtcm.F90:86
    nhbet: float = 0.4
    nhxkd: float = 0.1
    base_state_pressure: float = 101325.0
    logp_lrate: float = 47.70
    base_state_ts0: float = 288.15   # domain-file value in the reference; synthetic here

    def __post_init__(self):
        # dynparam defaults per core, Main/mod_params.F90:645-661
        if self.idynamic == 2:
            self.gnu1 = self.gnu2 = 0.1
            self.diffu_hgtf = 0
        # Share/mod_dynparam.F90:664-675
        for attr in ("nspgx", "nspgd"):
            if getattr(self, attr) is None:
                n = 12
                n = max(min(max(int(float(n * 50) / self.ds), n), min(self.jx, self.iy) // 4), 3)
                setattr(self, attr, max(n, 3))
        if self.kz not in SIGMA_TABLES:
            raise ValueError(f"no sigma table for kz={self.kz}")

    @property
    def nqx(self) -> int:
        """Moisture species: 5 (qv, qc, qi, qr, qs) for ipptls > 1, else 2 (qv, qc)."""
        return 5 if self.ipptls > 1 else 2

    @property
    def sigma(self) -> np.ndarray:
        return np.array(SIGMA_TABLES[self.kz], dtype=np.float64)

    @property
    def dtbdys(self) -> float:
        return float(self.ibdyfrq) * 3600.0


# BASELINE.json configs (C1..C4 hydrostatic; C5 needs the non-hydrostatic core).
CONFIGS = {
    "C1": RunConfig(jx=48, iy=48, kz=18, ds=60.0, dt=150.0, name="C1 48x48x18 test_001-like"),
    "C2": RunConfig(jx=96, iy=96, kz=23, ds=50.0, dt=100.0, name="C2 96x96x23 dt=100"),
    "C3": RunConfig(jx=192, iy=192, kz=23, ds=50.0, dt=150.0, name="C3 192x192x23 50km EURO"),
    "C4": RunConfig(jx=384, iy=384, kz=23, ds=50.0, dt=150.0, name="C4 384x384x23"),
    # non-hydrostatic: C5 is BASELINE's 3 km convection-permitting grid; N1/N2 are reduced
    # grids of the same core for parity tests.  dt = 9 s = 3 x ds(km), the reference's own
    # CFL rule of thumb (Doc/UserGuide/AdvancedConfig.tex:478-486; its only NH namelist,
    # PreProc/CRM/crm_test.in, runs 3 km at 5 s): SURVEY's 30 s diverges within 7 steps.
    "N1": RunConfig(jx=40, iy=36, kz=18, ds=3.0, dt=9.0, idynamic=2, name="N1 40x36x18 NH 3km"),
    "N2": RunConfig(jx=96, iy=96, kz=41, ds=3.0, dt=9.0, idynamic=2, name="N2 96x96x41 NH 3km"),
    "C5": RunConfig(jx=768, iy=768, kz=41, ds=3.0, dt=9.0, idynamic=2, name="C5 768x768x41 NH 3km"),
    # the reference's own non-hydrostatic namelist, PreProc/CRM/crm_test.in: 64x64x23 at 3 km,
    # dt 5 s, ptop 5 cb, i_band = 1 and i_crm = 1 (periodic in j and i, :16-17), iboudy = 0,
    # ibltyp = 2 (:81-82), idynamic = 2 (:123); every other option at its default
    "CRM": RunConfig(jx=64, iy=64, kz=23, ds=3.0, dt=5.0, idynamic=2, i_band=1, i_crm=1, iboudy=0, ibltyp=2,
                     name="CRM 64x64x23 NH 3km crm_test.in"),
}


def build_config(rc: RunConfig, split: dict, nproc_j: int = 1, nproc_i: int = 1,
                 tile_first: int = 0, tile_count: Optional[int] = None,
                 comm_rank: int = 0, comm_size: int = 1, device: int = -1,
                 unique_id: Optional[bytes] = None) -> RcmdynConfig:
    """Fill the C-ABI config from a RunConfig and the host-side vmodes/spinit constants."""
    c = RcmdynConfig()
    c.abi_version = ABI_VERSION
    c.jx, c.iy, c.kz = rc.jx, rc.iy, rc.kz
    c.nproc_j, c.nproc_i = nproc_j, nproc_i
    c.tile_first = tile_first
    c.tile_count = nproc_j * nproc_i if tile_count is None else tile_count
    c.idynamic = rc.idynamic
    c.iboudy, c.idiffu, c.ipgf, c.nsplit = rc.iboudy, rc.idiffu, rc.ipgf, rc.nsplit
    c.nspgx, c.nspgd = rc.nspgx, rc.nspgd
    c.diffu_hgtf = rc.diffu_hgtf
    c.upstream_mode = rc.upstream_mode
    c.stability_enhance = rc.stability_enhance
    c.present_qc = rc.present_qc
    c.ds, c.dtsec, c.ptop = rc.ds, rc.dt, rc.ptop
    c.gnu1, c.gnu2, c.uoffc = rc.gnu1, rc.gnu2, rc.uoffc
    c.t_extrema, c.q_rel_extrema = rc.t_extrema, rc.q_rel_extrema
    c.ckh, c.adyndif = rc.ckh, rc.adyndif
    c.high_nudge, c.medium_nudge, c.low_nudge = rc.high_nudge, rc.medium_nudge, rc.low_nudge
    c.bdy_nm, c.bdy_dm, c.dtbdys = rc.bdy_nm, rc.bdy_dm, rc.dtbdys
    sig = rc.sigma
    for k in range(rc.kz + 1):
        c.sigma[k] = sig[k]
    kz, ns = rc.kz, rc.nsplit
    for l in range(ns):
        for k in range(kz):
            c.zmatx[l][k] = split["zmatx"][k, l]
            c.zmatxr[l][k] = split["zmatxr"][l, k]
            c.am[l][k] = split["am"][k, l]
            c.tau[l][k] = split["tau"][l, k]
        for k in range(kz + 1):
            c.varpa1[l][k] = split["varpa1"][l, k]
        c.an[l] = split["an"][l]
        c.hbar[l] = split["hbar"][l]
        c.aam[l] = split["aam"][l]
        c.dtau[l] = split["dtau"][l]
    for k in range(kz + 1):
        c.sigmah[k] = split["sigmah"][k]
    c.pd = split["pd"]
    c.comm_rank, c.comm_size, c.device = comm_rank, comm_size, device
    if unique_id is not None:
        ctypes.memmove(c.comm_unique_id, unique_id, 128)
    c.ifupr, c.ifrayd, c.rayndamp = rc.ifupr, rc.ifrayd, rc.rayndamp
    c.nhbet, c.nhxkd, c.rayalpha0, c.rayhd = rc.nhbet, rc.nhxkd, rc.rayalpha0, rc.rayhd
    c.rhmin, c.rhmax = rc.rhmin, rc.rhmax
    c.isladvec, c.iqmsl = rc.isladvec, rc.iqmsl
    c.ibltyp, c.nuk, c.tkemin = rc.ibltyp, rc.nuk, rc.tkemin
    c.iuwvadv = rc.iuwvadv
    c.ipptls, c.nqx = rc.ipptls, rc.nqx
    c.i_band, c.i_crm, c.ichem = rc.i_band, rc.i_crm, rc.ichem
    if rc.idynamic == 2:
        c.nh_dtsmax = split["nh_dtsmax"]
        c.nh_xmsf = split["nh_xmsf"]
    return c


def set_nproc(nproc: int, jx: int, iy: int) -> Sequence[int]:
    """Decomposition rule of set_nproc, Main/mpplib/mod_mppparam.F90:1152-1186."""
    if nproc == 1:
        return (1, 1)
    if nproc < 4:
        return (nproc, 1)
    cj = (int(round(np.sqrt(float(nproc)))) // 2) * 2
    if iy > int(1.5 * float(jx)):
        cj -= 1
        while nproc % cj != 0:
            cj -= 1
    elif jx > int(1.5 * float(iy)):
        cj += 1
        while nproc % cj != 0:
            cj += 1
    else:
        while nproc % cj != 0:
            cj += 1
    return (cj, nproc // cj)

"""Algorithmic HBM bytes of the dyn-step kernels (the roofline numerators of bench.py).

"Algorithmic" = the compulsory traffic of a kernel: every field it must read or write,
counted once, at 8 bytes per fp64 value, over the points it updates.  Units are grid
points: N3 = jx*iy*kz (one 3-D field), N2 = jx*iy (one 2-D field); f_b is the fraction of
points in the boundary-relaxation band (the nudging kernels read b0/bt only there).
Whole-step total B_h is SURVEY.md section 8(d): 8 [N3 (20 + 8 f_b) + N2 (19 + 2 f_b)].

Per-kernel field counts (reads + writes of 3-D fields, 2-D fields) follow the kernels of
regcm_amd/csrc/kernels.hip with tendency diagnostics off:
  k_momentum    reads atm1 u,v,t,qv, atm2 u,v, qdot, xkc, phi (9) + u,v b0/bt in band (4 f_b);
                writes next atm1/atm2 u,v (4); 2-D: msfd msfx-derived dmsf coriol rpsa rpsda rpsdb
                psa psdota psdotb (9)
  k_scalars     reads atm1 u,v,t,qv,qc, atm2 u,v (xkc), atm2 t,qv,qc, qdot (11) + t,q b0/bt in
                band (4 f_b); writes next atm1/atm2 t, cqv, cqc and (qfuse, the RAW filter of
                the non-negative forecasts) next atm1/atm2 qv, qc (8); 2-D: 12 + psc
  k_update      k_momentum's and k_scalars' blocks in one launch: the union of their fields
                (the state both read counted once): reads atm1 u,v,t,qv,qc, atm2 u,v,t,qv,qc,
                qdot, xkc, phi (13) + u,v,t,q b0/bt in band (8 f_b); writes the 12 of the two;
                2-D: 14
  k_columns     reads atm1 u,v,t,qv,qc (5); writes qdot, phi (2); 2-D: 12 + (qfuse) the
                RA-filtered p* into the next buffers (2); the keep copies are O(perimeter)
  k_qfilter     (RCMDYN_NO_QFUSE) reads cqv,cqc, atm1/atm2 qv,qc (6); writes next atm1/atm2
                qv,qc (4); 2-D: 5
  k_split_project reads atm1/atm2 u,v,t (6); 2-D: 3 nsplit slots x 2 + 8
  k_split_correct read-modify-write atm1/atm2 t,u,v (12); 2-D: 2 nsplit + 4 (the bdyval blocks of
                k_split_correct_bdy move O(perimeter) more)
"""
from __future__ import annotations


def band_fraction(jx: int, iy: int, nspgx: int) -> float:
    return 1.0 - ((jx - 1 - 2 * nspgx) * (iy - 1 - 2 * nspgx)) / ((jx - 1) * (iy - 1))


# (3-D fields, 3-D fields in the band only, 2-D fields)
KERNEL_FIELDS = {
    "k_momentum": (13, 4, 9),
    "k_scalars": (19, 4, 13),
    "k_update": (25, 8, 14),
    "k_columns": (7, 0, 14),
    "k_qfilter": (10, 0, 5),
    "k_split_project": (6, 0, 20),
    "k_split_correct": (12, 0, 8),
    # non-hydrostatic core (kernels_nh.hip); 3-D fields of kz or kz+1 levels counted alike
    #   k_nh_sound_cd  reads se, sf, rhof0, cu, cv, pi, rho0, pr1, pp, ppten, atm2 qv, rho1,
    #                  atm2/atm1 t, pr0 (15); writes w, pp, pi, atm2/atm1 t, dp'/dp0 (6)
    #   k_nh_sound_bc  reads pp, pi, pr1, rho0, t0, pr0, atm2 t, ppten, cu, cv, rho1, w, wten (13);
    #                  writes se, sf, pi, pp (4)
    #   k_nh_tend_c    reads atm1 u, v, t, qv, qc, pp, w, atm2 t, qv, qc, pp, w, th, qdot, cr,
    #                  rho0, rho1, xpr, xkcr, z0, zf0 (21) + t, qv, pp, w b0/bt in the band
    #                  (8 f_b); writes wten, ppten, atmc qv, qc and the time-filtered atm1/atm2
    #                  t, qv, qc into the other parity (10; tfilter fused); the decoupled products
    #                  (xw, xpp, xqv, xqc, umc, vmc, the b-level fields, xkc, xkcf) are formed
    #                  from these as they are read
    #   k_nh_tend_d    reads atm1 u, v, w, atm2 u, v, ud, vd, cr, qdot, xkcr, z0 (11) + u, v b0/bt
    #                  in the band (4 f_b); writes uten, vten (2)
    "k_nh_sound_cd": (21, 0, 5),
    "k_nh_sound_bc": (17, 0, 6),
    "k_nh_tend_c": (31, 8, 9),
    "k_nh_tend_d": (13, 4, 10),
}


# level-marching forms of a kernel move the same fields (template arguments are stripped)
ALIASES = {"k_scalars_km": "k_scalars", "k_momentum_km": "k_momentum"}


def base_name(name: str) -> str:
    n = name.split("<")[0]
    return ALIASES.get(n, n)


def kernel_bytes(name: str, jx: int, iy: int, kz: int, nspgx: int) -> float | None:
    """Algorithmic bytes of one launch of `name` over a jx x iy x kz domain (None if the
    kernel has no entry)."""
    name = base_name(name)
    if name not in KERNEL_FIELDS:
        return None
    f3, fband, f2 = KERNEL_FIELDS[name]
    n3, n2 = jx * iy * kz, jx * iy
    fb = band_fraction(jx, iy, nspgx)
    return 8.0 * (n3 * (f3 + fband * fb) + n2 * f2)


def step_bytes(jx: int, iy: int, kz: int, nspgx: int) -> float:
    """SURVEY.md section 8(d) B_h: compulsory HBM bytes of one hydrostatic step."""
    n3, n2 = jx * iy * kz, jx * iy
    fb = band_fraction(jx, iy, nspgx)
    return 8.0 * (n3 * (20 + 8 * fb) + n2 * (19 + 2 * fb))


def step_bytes_nh(jx: int, iy: int, kz: int, nspgx: int, istep: int) -> float:
    """SURVEY.md section 8(d) B_nh: compulsory HBM bytes of one non-hydrostatic step,
    8 [N3 (34 + 12 f_b + 22 istep) + 21 N2]."""
    n3, n2 = jx * iy * kz, jx * iy
    fb = band_fraction(jx, iy, nspgx)
    return 8.0 * (n3 * (34 + 12 * fb + 22 * istep) + n2 * 21)

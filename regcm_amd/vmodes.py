"""Host-side initialisation of the split-explicit scheme: vertical modes + spinit constants.

This is init-only work that the reference does once on the host (``spinit``,
``Main/mod_split.F90:75-175`` -> ``vmodes``, ``Main/mod_vmodes.F90:86-594``).  The engine only
consumes its outputs through ``rcmdyn_config`` (out of scope for
the device).  The eigen-decomposition uses numpy/LAPACK instead of the vendored EISPACK ``rg``;
the column normalisation/ordering of ``vorder``/``vnorml`` makes the result unique.
"""
from __future__ import annotations

import math

import numpy as np

from . import constants as C


def vmodes(sigma: np.ndarray, ptop: float, kz: int) -> dict:
    """Restatement of vmodes with lstand = .true. (Main/mod_vmodes.F90:86-467)."""
    kzp1 = kz + 1
    sig = np.asarray(sigma, dtype=np.float64)          # 0-based: sig[k-1] = sigma(k)
    xps = C.stdpcb                                       # :149
    pd = xps - ptop                                      # :151
    sigmah = np.zeros(kzp1)
    sdsigma = np.zeros(kz)
    for k in range(kz):
        sigmah[k] = (sig[k] + sig[k + 1]) * 0.5          # :168-171
        sdsigma[k] = sig[k + 1] - sig[k]
    sigmah[kz] = 1.0
    # vtlaps :494-508
    tbarh = np.zeros(kz)
    fac = C.rgas * C.lrate * C.regrav
    for k in range(kz):
        p = sigmah[k] * pd + ptop
        tbarh[k] = C.stdt * ((p / C.stdpcb) ** fac)
        z = (C.stdt - tbarh[k]) / C.lrate
        if z > 10769.0:
            tbarh[k] = 218.15
    # thermodynamic matrix :182-262
    tbarf = np.zeros(kzp1)
    for k in range(1, kz):                               # Fortran k = 2..kz
        km1 = k - 1
        tbarf[k] = (tbarh[km1] * (sigmah[k] - sig[k]) / (sigmah[k] - sigmah[km1]) +
                    tbarh[k] * (sig[k] - sigmah[km1]) / (sigmah[k] - sigmah[km1]))
    e1 = np.ones((kz, kz))
    e2 = np.tril(np.ones((kz, kz)))                      # e2(k,l) = 1 for l <= k
    d1 = np.diag(sdsigma)
    a3 = np.diag(-tbarh)
    d2 = np.diag(C.rovcp * tbarh / (sigmah[:kz] + ptop / pd))
    s1 = np.diag(sig[:kz])
    s2 = np.diag(sigmah[:kz])
    x1 = np.eye(kz)
    e3 = np.eye(kz)
    g1 = np.zeros((kz, kz))
    for k in range(kz):
        if k > 0:
            g1[k, k] = tbarf[k]
        if k < kz - 1:
            g1[k, k + 1] = -tbarf[k + 1]
            e3[k, k + 1] = 1.0
    w1 = e2 - x1
    w2 = w1 @ d1
    g2 = e1 @ d1
    w1 = s1 @ g2
    g2 = w1 - w2
    w2 = np.diag(1.0 / sdsigma)
    a1 = w2 @ (g1 @ g2)
    a2 = s2 @ (e1 @ d1)
    w2 = (e3 @ g2) * 0.5
    a2 = d2 @ (w2 - a2)
    a4 = -(a3 @ (e1 @ d1))
    a0 = a1 + a2 + a3 + a4
    # hydrostatic matrices :270-310
    dlogp = np.zeros(kz)
    for k in range(1, kz):
        dlogp[k] = math.log((sigmah[k] + ptop / pd) / (sigmah[k - 1] + ptop / pd))
    hydros = np.zeros((kz, kz))
    for k in range(kz - 1):
        for l in range(k, kz - 1):
            hydros[k, l] += dlogp[l + 1] * sdsigma[l] / (sdsigma[l + 1] + sdsigma[l])
            hydros[k, l + 1] += dlogp[l + 1] * sdsigma[l + 1] / (sdsigma[l + 1] + sdsigma[l])
    for k in range(kz):
        hydros[k, kz - 1] += math.log((1.0 + ptop / pd) / (sigmah[kz - 1] + ptop / pd))
    hydroc = np.zeros((kz, kzp1))
    tweigh = np.zeros(kz)
    for l in range(1, kz):
        tweigh[l] = (tbarh[l] * sdsigma[l] + tbarh[l - 1] * sdsigma[l - 1]) / (sdsigma[l] + sdsigma[l - 1])
    for l in range(1, kz - 1):
        for k in range(l):
            hydroc[k, l] = tweigh[l] - tweigh[l + 1]
    for l in range(kz - 1):
        hydroc[l, l] = tbarh[l] - tweigh[l + 1]
    for k in range(kz - 1):
        hydroc[k, kz - 1] = tweigh[kz - 1] - tbarh[kz - 1]
    for k in range(kz):
        hydroc[k, kz] = tbarh[kz - 1]
    # tau :338-353
    w3 = np.zeros((kzp1, kz))
    for l in range(kz):
        for k in range(kzp1):
            w3[k, l] = sdsigma[l] / (1.0 + ptop / (pd * sigmah[k]))
    w2 = hydroc @ w3
    tau = -C.rgas * (hydros @ a0 - w2)
    # eigen-decomposition (rg) + vorder + vnorml :358-363
    evals, evecs = np.linalg.eig(tau)
    if np.max(np.abs(evals.imag)) > 1e-9 * np.max(np.abs(evals.real)):
        raise RuntimeError("vmodes: complex equivalent depths")
    evals = evals.real
    evecs = evecs.real
    order = np.argsort(-evals, kind="stable")
    hbar = evals[order]
    zmatx = evecs[:, order].copy()
    for l in range(kz):
        col = zmatx[:, l]
        kmax = int(np.argmax(np.abs(col)))
        zmax = abs(col[kmax])
        v = float(np.sum(sdsigma * col * col))
        a = (col[kmax] / zmax) / math.sqrt(v)
        zmatx[:, l] = a * col
    zmatxr = np.linalg.inv(zmatx)
    hydror = np.linalg.inv(hydros)
    # varpa1 :389-408
    hweigh = np.zeros(kz)
    hweigh[kz - 1] = 1.0
    w1 = np.zeros((kz, kz))
    for k1 in range(kz):
        for k2 in range(kz):
            s = 0.0
            for k in range(kz):
                s = hydror[k, k2] * hydror[k, k1] * hweigh[k] / (tbarh[k] ** 2) + s
            w1[k2, k1] = s
    varpa1 = (w1 @ hydroc) * (xps * xps)
    a0 = a0 - a4                                          # :422-426
    return dict(a0=a0, hbar=hbar, sigmah=sigmah, tbarh=tbarh, zmatx=zmatx, zmatxr=zmatxr,
                tau=tau, varpa1=varpa1, hydroc=hydroc, hydros=hydros, pd=pd, xps=xps)


def spinit_constants(sigma: np.ndarray, ptop: float, kz: int, dtsec: float, nsplit: int) -> dict:
    """The mode constants spinit leaves in mod_split (Main/mod_split.F90:86-175)."""
    vm = vmodes(sigma, ptop, kz)
    dsigma = np.diff(np.asarray(sigma, dtype=np.float64))
    dtau = np.array([dtsec * (0.5 / float(nsplit - ns)) for ns in range(nsplit)])  # mod_params:1703-1706
    aam = np.array([float(int(math.floor(dtsec / dtau[ns] + 0.5))) for ns in range(nsplit)])
    zmatx = vm["zmatx"].copy()
    zmatxr = vm["zmatxr"]
    a0, hydros, hydroc = vm["a0"], vm["hydros"], vm["hydroc"]
    an = np.zeros(nsplit)
    am = np.zeros((kz, nsplit))
    tau = vm["tau"].copy()
    varpa1 = vm["varpa1"].copy()
    for n in range(nsplit):
        s = 0.0
        for l in range(kz):
            s = s + dsigma[l] * zmatx[l, n]
        an[n] = s
        for k in range(kz):
            am[k, n] = 0.0
            tau[n, k] = 0.0
        for l in range(kz):
            for k in range(kz):
                am[k, n] = am[k, n] + a0[k, l] * zmatx[l, n]
                tau[n, k] = tau[n, k] + C.rgas * zmatxr[n, l] * hydros[l, k]
        for k in range(kz + 1):
            varpa1[n, k] = 0.0
        for l in range(kz):
            for k in range(kz + 1):
                varpa1[n, k] = varpa1[n, k] + C.rgas * zmatxr[n, l] * hydroc[l, k]
    for l in range(nsplit):
        fac = 2.0 * dtsec / (2.0 * aam[l] + 1.0)
        an[l] = an[l] * fac
        zmatx[:, l] = zmatx[:, l] * fac
        am[:, l] = am[:, l] * fac
    return dict(zmatx=zmatx, zmatxr=zmatxr, am=am, an=an, tau=tau, varpa1=varpa1,
                hbar=vm["hbar"], aam=aam, dtau=dtau, sigmah=vm["sigmah"], pd=vm["pd"])

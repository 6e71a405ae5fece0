"""CPU oracle for the LDPC side of the joint decoder.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
checker: the product (``sparc_ldpc_amd``) never calls it.

A NumPy restatement of the reference's LDPC code class and C decoders:

* protograph -> Tanner graph (vdeg, cdeg, intrlv)   ldpc/py/ldpc.py:694-786
* systematic QC encoder                             ldpc/py/ldpc.py:790-850
* parity-check matrix                               ldpc/py/ldpc.py:666-691
* sumprod / sumprod2 / minsum flooding decoders     ldpc/src/c_ldpc.c:32-113, 138-206, 339-381
* Lxor / Lxfb                                       ldpc/src/c_ldpc.c:234-251, 294-314
* sp2bp / bp2sp / LLR glue                          ldpc/sparc_ldpc.py:257-314, 470-479

Every per-node operation runs in the reference's order (same additions, same
Lxor association), vectorised across nodes of equal degree, so results agree
with the reference C decoder up to the last-ulp differences between NumPy's
and glibc's exp/log.  Pinned by ``tests/golden/ldpc.npz`` (reference graphs,
encoder and C-decoder KATs; ``tests/test_ldpc_oracle.py``) and, when
``oracle/_ref/c_ldpc.so`` has been built from the reference's own source by
``oracle/Makefile``, against that library directly.

One deliberate difference: the reference ``minsum`` advances its message
offset by ``cdeg[j+1]`` instead of ``cdeg[j]`` (c_ldpc.c:364), which only
agrees with the intended rule for check-regular codes; this restatement (and
the HIP decoder) use the aligned offsets, and minsum parity is asserted on
check-regular codes only.
"""
from __future__ import annotations

import json
import os

import numpy as np

MAX_ITCOUNT = 200  # c_ldpc.c:7
_DATA = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                     "sparc_ldpc_amd", "data", "protographs.json")


def protograph(standard, rate, z, ptype="A"):
    """Base matrix of ldpc.py:26-663 (data captured from the reference)."""
    with open(_DATA) as fh:
        tab = json.load(fh)["protographs"]
    if standard == "802.11n":
        return np.array(tab["802.11n"][str(z)][rate], dtype=np.int64)
    return np.array(tab["z_free"][standard][rate][ptype], dtype=np.int64)


def prepare_decoder(proto, z):
    """ldpc.py:694-786: ports are taken in protograph row-major order, so a
    check node's ports follow its row's columns and a variable node's ports
    follow its column's rows."""
    proto = np.asarray(proto)
    cdeg = np.repeat(np.sum(proto != -1, 1), z)
    vdeg = np.repeat(np.sum(proto != -1, 0), z)
    cumc = np.concatenate([[0], np.cumsum(cdeg)])
    cumv = np.concatenate([[0], np.cumsum(vdeg)])
    nmsg = int(cumc[-1])
    intrlv = np.empty(nmsg, dtype=np.int64)
    mask = proto != -1
    rank_row = np.cumsum(mask, 1) - 1  # port of (xp, yp) inside check nodes of row xp
    rank_col = np.cumsum(mask, 0) - 1  # port of (xp, yp) inside variable nodes of column yp
    k = np.arange(z)
    for xp, yp in zip(*np.nonzero(mask)):
        off = proto[xp, yp]
        cind = xp * z + k
        vind = yp * z + (k + off) % z
        intrlv[cumv[vind] + rank_col[xp, yp]] = cumc[cind] + rank_row[xp, yp]
    return vdeg.astype(np.int64), cdeg.astype(np.int64), intrlv


def pcmat(proto, z):
    """ldpc.py:666-691."""
    proto = np.asarray(proto)
    H = np.zeros((z * proto.shape[0], z * proto.shape[1]), dtype=np.int64)
    for r, c in zip(*np.nonzero(proto != -1)):
        H[r * z:(r + 1) * z, c * z:(c + 1) * z] = np.roll(np.eye(z, dtype=np.int64), proto[r, c] % z, 1)
    return H


def encode(proto, z, info):
    """ldpc.py:790-850 (one information word)."""
    proto = np.asarray(proto)
    Mp, Np = proto.shape
    Kp = Np - Mp
    info = np.asarray(info, dtype=np.int64)
    if info.size != Kp * z:
        raise NameError("information word length not compatible with proto and z")
    x = np.zeros((Np, z), dtype=np.int64)
    x.reshape(-1)[:Kp * z] = info
    p = np.zeros((Mp, z), dtype=np.int64)
    for j in range(Mp):
        for k in np.nonzero(proto[j, :Kp] != -1)[0]:
            p[j] += np.roll(x[k], -proto[j, k])
    p %= 2
    tp = p.sum(0) % 2
    toff = np.zeros(z, dtype=np.int64)
    for j in np.nonzero(proto[:, Kp] != -1)[0]:
        toff[proto[j, Kp] % z] += 1
    tnz = np.nonzero(toff % 2)[0]
    if len(tnz) != 1:
        raise NameError("The offsets in colum Kp+1 of proto do not add to a single offset")
    x[Kp] = np.roll(tp, tnz[0])
    for j in range(Mp - 1):
        myk = Kp + j + 1
        x[myk] = p[j]
        for k in np.nonzero(proto[j, Kp:myk] != -1)[0]:
            x[myk] += np.roll(x[Kp + k], -proto[j, Kp + k])
    return (x % 2).reshape(-1)


# ---- decoders ---------------------------------------------------------------

def lxor(L1, L2, corr=True):
    """c_ldpc.c:234-251, elementwise."""
    s = np.where(np.signbit(L1) == np.signbit(L2), 1.0, -1.0)
    L = s * np.fmin(np.abs(L1), np.abs(L2))
    if corr:
        with np.errstate(over="ignore", invalid="ignore"):
            L = L + np.log(1 + np.exp(-np.abs(L1 + L2)))
            L = L - np.log(1 + np.exp(-np.abs(L1 - L2)))
    return L


def lxfb(Lm, corr=True):
    """c_ldpc.c:294-314 on the rows of Lm (n_nodes x dc), in place; returns b[0]."""
    dc = Lm.shape[1]
    f = [None] * dc
    b = [None] * dc
    f[0] = Lm[:, 0].copy()
    b[dc - 1] = Lm[:, dc - 1].copy()
    for k in range(1, dc):
        f[k] = lxor(f[k - 1], Lm[:, k], corr)
        b[dc - k - 1] = lxor(b[dc - k], Lm[:, dc - k - 1], corr)
    Lm[:, 0] = b[1]
    Lm[:, dc - 1] = f[dc - 2]
    for k in range(1, dc - 1):
        Lm[:, k] = lxor(f[k - 1], b[k + 1], corr)
    return b[0]


class _Graph:
    def __init__(self, vdeg, cdeg, intrlv):
        self.vdeg = np.asarray(vdeg, np.int64)
        self.cdeg = np.asarray(cdeg, np.int64)
        self.intrlv = np.asarray(intrlv, np.int64)
        cumv = np.concatenate([[0], np.cumsum(self.vdeg)])
        cumc = np.concatenate([[0], np.cumsum(self.cdeg)])
        self.vgroups = []  # (nodes, edge matrix of message indices) per degree
        for d in np.unique(self.vdeg):
            nodes = np.nonzero(self.vdeg == d)[0]
            E = self.intrlv[cumv[nodes][:, None] + np.arange(d)[None, :]]
            self.vgroups.append((nodes, E))
        self.cgroups = []
        for d in np.unique(self.cdeg):
            nodes = np.nonzero(self.cdeg == d)[0]
            E = cumc[nodes][:, None] + np.arange(d)[None, :]
            self.cgroups.append((nodes, E))


def _decode(ch, vdeg, cdeg, intrlv, algo, corr_factor=0.7, max_it=MAX_ITCOUNT):
    g = _Graph(vdeg, cdeg, intrlv)
    ch = np.asarray(ch, dtype=np.float64)
    msg = np.zeros(len(g.intrlv))
    app = np.zeros(len(g.vdeg))
    it = 0
    with np.errstate(over="ignore", invalid="ignore", divide="ignore"):
        for it in range(max_it):
            # variable nodes (c_ldpc.c:171-178): sequential sum in port order
            for nodes, E in g.vgroups:
                aggr = ch[nodes].copy()
                for k in range(E.shape[1]):
                    aggr = aggr + msg[E[:, k]]
                old = msg[E]
                msg[E] = aggr[:, None] - old
                app[nodes] = aggr
            unsat = False
            for nodes, E in g.cgroups:
                Lm = msg[E]
                if algo == "sumprod":  # c_ldpc.c:76-102
                    Lm = np.tanh(Lm / 2.0)
                    aggr = np.ones(len(nodes))
                    for k in range(Lm.shape[1]):
                        aggr = aggr * Lm[:, k]
                    unsat |= bool(np.any(2.0 * np.arctanh(aggr) <= 0.0))
                    Lm = 2.0 * np.arctanh(aggr[:, None] / Lm)
                elif algo == "sumprod2":
                    aggr = lxfb(Lm, True)
                    unsat |= bool(np.any(aggr <= 0.0))
                elif algo == "minsum":
                    aggr = lxfb(Lm, False)
                    unsat |= bool(np.any(aggr <= 0.0))
                    Lm = Lm * corr_factor
                else:
                    raise NameError("Decoder type unknonwn")
                msg[E] = Lm
            if not unsat:
                return app, it
    return app, max_it


def sumprod2(ch, vdeg, cdeg, intrlv):
    return _decode(ch, vdeg, cdeg, intrlv, "sumprod2")


def sumprod(ch, vdeg, cdeg, intrlv):
    return _decode(ch, vdeg, cdeg, intrlv, "sumprod")


def minsum(ch, vdeg, cdeg, intrlv, corr_factor=0.7):
    return _decode(ch, vdeg, cdeg, intrlv, "minsum", corr_factor)


# ---- SPARC <-> bits glue ---------------------------------------------------------

def sp2bp(beta, L, M):
    """sparc_ldpc.py:257-281: p[b] = P(bit b == 1); section bits MSB first."""
    logm = int(np.log2(M))
    p = np.zeros(logm * L)
    beta = np.asarray(beta, dtype=np.float64).reshape(-1)
    for a in range(L):
        bl = beta[a * M:(a + 1) * M]
        for logi in range(logm):
            b = (a + 1) * logm - logi - 1
            i = 2 ** logi
            k = i
            while k < M:
                for j in range(k, k + i):
                    p[b] = p[b] + bl[j]
                k += 2 * i
    return p


def bp2sp(v, L, M):
    """sparc_ldpc.py:283-314 (product of independent bit marginals, normalised)."""
    logm = int(np.log2(M))
    v = np.asarray(v, dtype=np.float64)
    sp = np.zeros(L * M)
    for l in range(L):
        bp = v[l * logm:(l + 1) * logm]
        for m in range(M):
            bits = np.array([int(c) for c in bin(m)[2:].zfill(logm)])
            a = bp ** bits
            b = (1 - bp) ** (1 - bits)
            sp[l * M + m] = np.prod(a * b)
        sp[l * M:(l + 1) * M] = sp[l * M:(l + 1) * M] / sum(sp[l * M:(l + 1) * M])
    return sp


def llr_from_beta(beta, Pl, n, L, M, nsec):
    """sparc_ldpc.py:470-479 for the last ``nsec`` sections."""
    beta = np.asarray(beta, dtype=np.float64).reshape(-1)
    post = beta / np.sqrt(n * np.repeat(np.asarray(Pl, dtype=np.float64), M))
    p = sp2bp(post[(L - nsec) * M:], nsec, M)
    with np.errstate(divide="ignore"):
        llr = np.log(1 - p) - np.log(p)
    return np.nan_to_num(llr)

"""Independent Python restatement of CpGIslandFinder's hot path.

TEST INFRASTRUCTURE ONLY — the second, independent CPU restatement that the C oracle
(oracle/cpg_oracle.c) is cross-checked against on small inputs (pure-Python loops:
keep T small).  Never imported by the product package.

PARITY UNPINNED: the Java reference cannot run here and ships no tests.
Citations are to /root/reference/CpGIslandFinder.java.
"""
from __future__ import annotations

import math
import struct

import numpy as np

DBL_MAX = 1.7976931348623157e308

# CpGIslandFinder.java:155-173
INITIAL_PI = [0.05, 0.05, 0.05, 0.05, 0.2, 0.2, 0.2, 0.2]
INITIAL_A = [
    [0.170, 0.274, 0.426, 0.120, 0.0025, 0.0025, 0.0025, 0.0025],
    [0.170, 0.358, 0.274, 0.188, 0.0025, 0.0025, 0.0025, 0.0025],
    [0.161, 0.329, 0.375, 0.125, 0.0025, 0.0025, 0.0025, 0.0025],
    [0.079, 0.345, 0.384, 0.182, 0.0025, 0.0025, 0.0025, 0.0025],
    [0.0025, 0.0025, 0.0025, 0.0025, 0.300, 0.205, 0.275, 0.210],
    [0.0025, 0.0025, 0.0025, 0.0025, 0.393, 0.137, 0.088, 0.372],
    [0.0025, 0.0025, 0.0025, 0.0025, 0.248, 0.246, 0.288, 0.208],
    [0.0025, 0.0025, 0.0025, 0.0025, 0.177, 0.239, 0.282, 0.292],
]
INITIAL_B = [[1.0 if k == i % 4 else 0.0 for k in range(4)] for i in range(8)]

SYM = {ord("A"): 0, ord("a"): 0, ord("C"): 1, ord("c"): 1,
       ord("G"): 2, ord("g"): 2, ord("T"): 3, ord("t"): 3}


def _log(x: float) -> float:
    return math.log(x) if x > 0 else (-math.inf if x == 0 else math.nan)


def ingest(txt: bytes, chunk: int, count0: int = 0):
    """:112-145 (chunk=0x10000) / :238-259 (chunk=0x100000), quirk-faithful.

    Returns (list of chunks as lists of symbols, crash_flag).  For the training chunk
    size an empty list at a chunk multiple yields an all-zero chunk (new DenseVector);
    for the decode size it is the reference's crash (get(i) on an empty list).
    `count` is a Java int: at 2^32 it wraps to 0 and the test is skipped, so the list keeps
    its chunk and grows; at the next multiple the training reader's DenseVector.set(65536)
    throws (crash), the decode reader copies get(0 .. 2^20-1) and clear() drops the rest.
    count0 = the Java count before the first byte (test hook; a multiple of `chunk`)."""
    count = count0 & 0xFFFFFFFF
    lst: list[int] = []
    chunks = []
    for ch in txt:
        v = SYM.get(ch, -1)
        if v != -1:
            lst.append(v)
            count = (count + 1) & 0xFFFFFFFF
        if count != 0 and count % chunk == 0:
            if chunk == 0x100000 and len(lst) < chunk:
                return chunks, True                 # get(i) on an empty list
            if chunk == 0x10000 and len(lst) > chunk:
                return chunks, True                 # DenseVector(0x10000).set(0x10000, ...)
            c = [0] * chunk
            c[: min(len(lst), chunk)] = lst[:chunk]
            chunks.append(c)
            lst = []
    return chunks, False


def viterbi8(pi, a, b, obs):
    """Mahout HmmAlgorithms.viterbiAlgorithm(scaled=true) (called at :260)."""
    T = len(obs)
    delta = [_log(pi[i] * b[i][obs[0]]) for i in range(8)]
    phi = []
    for t in range(1, T):
        nd, row = [0.0] * 8, [0] * 8
        for i in range(8):
            ms, mp = 0, delta[0] + _log(a[0][i])     # Mahout: candidate 0 first (A.2)
            for j in range(1, 8):
                p = delta[j] + _log(a[j][i])
                if p > mp:
                    mp, ms = p, j
            nd[i] = mp + _log(b[i][obs[t]])
            row[i] = ms
        phi.append(row)
        delta = nd
    seq = [0] * T
    mp = -math.inf
    for i in range(8):
        if delta[i] > mp:
            mp, seq[T - 1] = delta[i], i
    for t in range(T - 2, -1, -1):
        seq[t] = phi[t][seq[t + 1]]
    return seq, mp


def estep8(pi, a, b, obs):
    """Rabiner-rescaled forward-backward; returns (init, trans, emit,
    loglik) for one sequence, in the same operation order as the C oracle."""
    T = len(obs)
    al = []
    c = []
    x = [pi[i] * b[i][obs[0]] for i in range(8)]
    s = 0.0
    for v in x:
        s += v
    c.append(1.0 / s)
    al.append([v * c[0] for v in x])
    for t in range(1, T):
        ap = al[-1]
        at = []
        s = 0.0
        for j in range(8):
            acc = 0.0
            for i in range(8):
                acc += ap[i] * a[i][j]
            at.append(acc * b[j][obs[t]])
            s += at[j]
        c.append(1.0 / s)
        al.append([v * c[t] for v in at])
    ll = 0.0
    for v in c:
        ll -= math.log(v)
    init = [0.0] * 8
    trans = [[0.0] * 8 for _ in range(8)]
    emit = [[0.0] * 4 for _ in range(8)]
    bc = [1.0] * 8
    for t in range(T - 1, -1, -1):
        at = al[t]
        den = 0.0
        for k in range(8):
            den += at[k] * bc[k]
        for i in range(8):
            g = (at[i] * bc[i]) / den
            emit[i][obs[t]] += g
            if t == 0:
                init[i] += g
        if t == 0:
            break
        ap = al[t - 1]
        num = [[((ap[i] * a[i][j]) * b[j][obs[t]]) * bc[j] for j in range(8)] for i in range(8)]
        dx = 0.0
        for i in range(8):
            for j in range(8):
                dx += num[i][j]
        for i in range(8):
            for j in range(8):
                trans[i][j] += num[i][j] / dx
        bn = []
        for i in range(8):
            acc = 0.0
            for j in range(8):
                acc += (a[i][j] * b[j][obs[t]]) * bc[j]
            bn.append(acc * c[t])
        bc = bn
    return init, trans, emit, ll


def count_labelled(obs: np.ndarray, sign: np.ndarray, chunk_len: int):
    """Build-defined labelled counts, numpy, over whole chunks."""
    n = (len(obs) // chunk_len) * chunk_len
    o = obs[:n].astype(np.int64).reshape(-1, chunk_len)
    s = o + np.where(sign[:n].reshape(-1, chunk_len) != 0, 0, 4)
    init = np.bincount(s[:, 0], minlength=8)
    trans = np.bincount((s[:, :-1] * 8 + s[:, 1:]).ravel(), minlength=64).reshape(8, 8)
    emit = np.bincount((s * 4 + o).ravel(), minlength=32).reshape(8, 4)
    dinuc = np.bincount((o[:, :-1] * 4 + o[:, 1:]).ravel(), minlength=16).reshape(4, 4)
    mono = np.bincount(o.ravel(), minlength=4)
    return init, trans, emit, dinuc, mono


def _i32(x: int) -> int:
    x &= 0xFFFFFFFF
    return x - (1 << 32) if x >= (1 << 31) else x


def islands(states, chunk: int):
    """CpGIslandFinder.java:262-339, literal transcription (Java int wrap via _i32)."""
    out = []
    beg = 0
    in_island = False
    c_count = g_count = cg_count = island_len = 0
    at_c = False
    for i, val in enumerate(states):
        if in_island:
            if val in (4, 5, 6, 7):
                in_island = False
                end = i - 1
                ccnt, gcnt = float(c_count), float(g_count)
                cg = (ccnt + gcnt) / island_len
                oe = 0.0
                if c_count != 0 and g_count != 0:
                    oe = _i32(cg_count * island_len) / (ccnt * gcnt)
                if cg > 0.5 and oe > 0.6:
                    out.append((_i32(beg + _i32(chunk * len(states)) + 1),
                                _i32(end + _i32(chunk * len(states)) + 1),
                                island_len, cg, oe))
            else:
                island_len += 1
                if val == 2:
                    g_count += 1
                    if at_c:
                        cg_count += 1
                if val == 1:
                    c_count += 1
                    at_c = True
                else:
                    at_c = False
        else:
            if val in (0, 1, 2, 3):
                in_island = True
                island_len = 1
                cg_count = 0
                beg = i
                if val == 1:
                    c_count = 1
                    at_c = True
                else:
                    c_count = 0
                g_count = 1 if val == 2 else 0
    return out


def java_f6(x: float) -> str:
    """java.util.Formatter '%f': shortest round-trip digits (repr), HALF_UP to 6."""
    from decimal import ROUND_HALF_UP, Decimal
    x = float(x)
    return str(Decimal(repr(x)).quantize(Decimal("0.000001"), rounding=ROUND_HALF_UP))


def java_dtoa(x: float) -> str:
    """java.lang.Double.toString (JDK 19+ spec: shortest round-trip digits, `repr`'s):
    plain decimal for 1e-3 <= |x| < 1e7 with at least one fraction digit, else
    d.ddd...E[-]n.  Used for the trained-model file of CpGIslandFinder.java:207-224."""
    import math
    from decimal import Decimal
    x = float(x)
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    sign = "-" if math.copysign(1.0, x) < 0 else ""
    if x == 0.0:
        return sign + "0.0"
    t = Decimal(repr(abs(x))).as_tuple()
    digits = "".join(map(str, t.digits)).rstrip("0") or "0"
    e = t.exponent + len(t.digits)            # value = 0.digits x 10^e
    if 1e-3 <= abs(x) < 1e7:
        if e > 0:
            ip = (digits + "0" * e)[:e]
            fp = digits[e:]
        else:
            ip, fp = "0", "0" * (-e) + digits
        return sign + ip + "." + (fp or "0")
    return sign + digits[0] + "." + (digits[1:] or "0") + "E" + str(e - 1)


def format_model(m) -> str:
    """The trained-model file (:207-224) for a 104-double model pi|a|b."""
    import numpy as np
    m = np.asarray(m, np.float64)
    pi, a, b = m[:8], m[8:72].reshape(8, 8), m[72:104].reshape(8, 4)
    out = []
    for i in range(8):
        out.append(java_dtoa(pi[i]) + "\n")
        out.append("".join(java_dtoa(v) + " " for v in a[i]) + "\n")
        out.append("".join(java_dtoa(v) + " " for v in b[i]) + "\n")
    return "".join(out)


def format_island(rec) -> str:
    beg, end, ln, cg, oe = rec
    return "%d %d %d %s %s\n" % (beg, end, ln, java_f6(cg), java_f6(oe))


def pack(obs: np.ndarray) -> np.ndarray:
    """2-bit pack, 16 bases per uint32, base k at bits 2*(k%16)."""
    n = len(obs)
    w = (n + 15) // 16
    pad = np.zeros(w * 16, dtype=np.uint32)
    pad[:n] = obs
    sh = (np.arange(16, dtype=np.uint32) * 2)[None, :]
    return (pad.reshape(w, 16) << sh).sum(axis=1, dtype=np.uint64).astype(np.uint32)


def unpack(packed: np.ndarray, n: int) -> np.ndarray:
    sh = (np.arange(16, dtype=np.uint32) * 2)[None, :]
    return ((packed.astype(np.uint32)[:, None] >> sh) & 3).astype(np.uint8).ravel()[:n]


def pack_bits(bits: np.ndarray) -> np.ndarray:
    n = len(bits)
    w = (n + 31) // 32
    pad = np.zeros(w * 32, dtype=np.uint64)
    pad[:n] = bits != 0
    sh = np.arange(32, dtype=np.uint64)[None, :]
    return (pad.reshape(w, 32) << sh).sum(axis=1, dtype=np.uint64).astype(np.uint32)


def unpack_bits(words: np.ndarray, n: int) -> np.ndarray:
    sh = np.arange(32, dtype=np.uint32)[None, :]
    return ((words.astype(np.uint32)[:, None] >> sh) & 1).astype(np.uint8).ravel()[:n]


def f64_bits(x: float) -> int:
    return struct.unpack("<Q", struct.pack("<d", x))[0]

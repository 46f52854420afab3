"""ctypes loader for the oracle — TEST INFRASTRUCTURE ONLY.

Two libraries:

* ``_build/liboracle.so``: the CPU restatement (delta_oracle.c) of the
  reference's src/c algorithms.  It is the checker for the HIP path.
* ``_ref/libdelta_ref.so``: the reference's own src/c sources compiled by
  oracle/Makefile (only where /root/reference exists; the built .so travels to
  the GPU box).  Used to pin the restatement.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  The product (delta-compression_amd/) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
_ORACLE_SO = os.path.join(HERE, "_build", "liboracle.so")
_REF_SO = os.path.join(HERE, "_ref", "libdelta_ref.so")
REF_BENCH = os.path.join(HERE, "_ref", "ref_bench")
REF_CLI = os.path.join(HERE, "_ref", "delta")

ONEPASS = 1
CORRECTING = 2
SEED_LEN = 16
TABLE_SIZE = 1048573
BUF_CAP = 256
MAX_TABLE = 1073741827


def build(ref: bool = False) -> None:
    targets = ["all"] + (["ref"] if ref else [])
    subprocess.run(["make", "-s", "-C", HERE] + targets, check=True)


class _Cmd(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("pad", C.c_uint32), ("r_off", C.c_uint64),
                ("v_off", C.c_uint64), ("len", C.c_uint64)]


def _buf(b: bytes):
    return C.cast(C.c_char_p(b), C.POINTER(C.c_uint8)) if b else None


class Oracle:
    def __init__(self, path: str = _ORACLE_SO):
        if not os.path.exists(path):
            build()
        L = self.L = C.CDLL(path)
        u8p, u64, sz = C.POINTER(C.c_uint8), C.c_uint64, C.c_size_t
        L.or_crc64_xz_u64.restype = u64
        L.or_crc64_xz_u64.argtypes = [u8p, sz]
        L.or_next_prime.restype = u64
        L.or_next_prime.argtypes = [u64]
        L.or_is_prime.restype = C.c_int
        L.or_is_prime.argtypes = [u64]
        L.or_onepass_q.restype = u64
        L.or_onepass_q.argtypes = [u64, u64, u64]
        L.or_fingerprint.restype = u64
        L.or_fingerprint.argtypes = [u8p, sz, sz]
        L.or_mod_mersenne.restype = u64
        L.or_mod_mersenne.argtypes = [u64, u64]
        L.or_correcting_params.argtypes = [u64, u64, u64, u64, C.POINTER(u64), C.POINTER(u64), C.POINTER(u64)]
        L.or_diff_onepass.restype = sz
        L.or_diff_onepass.argtypes = [u8p, sz, u8p, sz, sz, sz, C.POINTER(C.POINTER(_Cmd))]
        L.or_diff_correcting.restype = sz
        L.or_diff_correcting.argtypes = [u8p, sz, u8p, sz, sz, sz, sz, sz, C.POINTER(C.POINTER(_Cmd))]
        L.or_encode_pair.restype = sz
        L.or_encode_pair.argtypes = [C.c_int, u8p, sz, u8p, sz, sz, sz, sz, sz, C.POINTER(u8p)]
        L.or_decode_apply.restype = C.c_int
        L.or_decode_apply.argtypes = [u8p, sz, u8p, sz, C.c_int, C.POINTER(u8p), C.POINTER(sz)]
        L.or_synth_random.argtypes = [u64, u8p, sz]
        L.or_synth_edits.argtypes = [u64, u8p, sz, u64]
        L.or_synth_transpose.restype = sz
        L.or_synth_transpose.argtypes = [u64, C.c_uint32, C.c_uint32, C.c_uint32, u8p, u8p, sz]
        L.or_synth_shift.restype = sz
        L.or_synth_shift.argtypes = [u64, sz, u64, C.c_uint32, u8p, u8p]
        L.or_splitmix64_at.restype = u64
        L.or_splitmix64_at.argtypes = [u64, u64]
        L.or_free.argtypes = [C.c_void_p]

    # -- primitives ---------------------------------------------------------
    def crc64_xz(self, data: bytes) -> bytes:
        return self.L.or_crc64_xz_u64(_buf(data), len(data)).to_bytes(8, "big")

    def next_prime(self, n: int) -> int:
        return self.L.or_next_prime(n)

    def is_prime(self, n: int) -> bool:
        return bool(self.L.or_is_prime(n))

    def onepass_q(self, r_len: int, p: int = SEED_LEN, q: int = TABLE_SIZE) -> int:
        return self.L.or_onepass_q(r_len, p, q)

    def correcting_params(self, r_len: int, p: int = SEED_LEN, q: int = TABLE_SIZE,
                          max_table: int = MAX_TABLE):
        a, b, c = C.c_uint64(), C.c_uint64(), C.c_uint64()
        self.L.or_correcting_params(r_len, p, q, max_table, C.byref(a), C.byref(b), C.byref(c))
        return a.value, b.value, c.value

    def fingerprint(self, data: bytes, off: int, p: int) -> int:
        return self.L.or_fingerprint(_buf(data), off, p)

    def mod_mersenne(self, x: int) -> int:
        return self.L.or_mod_mersenne(x >> 64, x & (2**64 - 1))

    # -- algorithms ---------------------------------------------------------
    def _cmds(self, ptr, n):
        out = []
        for i in range(n):
            c = ptr[i]
            if c.kind == 1:
                out.append(("COPY", c.v_off, c.r_off, c.len))
            else:
                out.append(("ADD", c.v_off, c.len))
        self.L.or_free(ptr)
        return out

    def diff_onepass(self, R: bytes, V: bytes, p: int = SEED_LEN, q: int = TABLE_SIZE):
        ptr = C.POINTER(_Cmd)()
        n = self.L.or_diff_onepass(_buf(R), len(R), _buf(V), len(V), p, q, C.byref(ptr))
        return self._cmds(ptr, n)

    def diff_correcting(self, R: bytes, V: bytes, p: int = SEED_LEN, q: int = TABLE_SIZE,
                        buf_cap: int = BUF_CAP, max_table: int = MAX_TABLE):
        ptr = C.POINTER(_Cmd)()
        n = self.L.or_diff_correcting(_buf(R), len(R), _buf(V), len(V), p, q, buf_cap,
                                      max_table, C.byref(ptr))
        return self._cmds(ptr, n)

    def encode(self, algo: int, R: bytes, V: bytes, p: int = SEED_LEN, q: int = TABLE_SIZE,
               buf_cap: int = BUF_CAP, max_table: int = MAX_TABLE) -> bytes:
        out = C.POINTER(C.c_uint8)()
        n = self.L.or_encode_pair(algo, _buf(R), len(R), _buf(V), len(V), p, q, buf_cap,
                                  max_table, C.byref(out))
        res = C.string_at(out, n)
        self.L.or_free(out)
        return res

    def decode(self, R: bytes, delta: bytes, ignore_hash: bool = False):
        out = C.POINTER(C.c_uint8)()
        n = C.c_size_t()
        rc = self.L.or_decode_apply(_buf(R), len(R), _buf(delta), len(delta),
                                    int(ignore_hash), C.byref(out), C.byref(n))
        if rc != 0:
            return rc, None
        res = C.string_at(out, n.value) if n.value else b""
        self.L.or_free(out)
        return 0, res

    # -- synthetic workloads -----------------------------------------------
    def synth_random(self, seed: int, n: int) -> bytes:
        b = (C.c_uint8 * max(n, 1))()
        self.L.or_synth_random(seed, b, n)
        return bytes(b)[:n]

    def synth_pair(self, seed: int, n: int, n_edits: int):
        b = (C.c_uint8 * max(n, 1))()
        self.L.or_synth_random(seed, b, n)
        R = bytes(b)[:n]
        self.L.or_synth_edits(seed, b, n, n_edits)
        return R, bytes(b)[:n]

    def synth_transpose(self, seed: int, num_blocks: int, mean: int, pct: int = 50):
        cap = num_blocks * (mean * 3 // 2 + 1)
        r = (C.c_uint8 * cap)()
        v = (C.c_uint8 * cap)()
        n = self.L.or_synth_transpose(seed, num_blocks, mean, pct, r, v, cap)
        return bytes(r)[:n], bytes(v)[:n]

    def synth_shift(self, seed: int, n: int, n_edits: int, indel_pct: int):
        """Shift pair (substitutions, insertions and deletions; or_synth_shift)."""
        r = (C.c_uint8 * max(n, 1))()
        v = (C.c_uint8 * max(n + 8 * n_edits, 1))()
        m = self.L.or_synth_shift(seed, n, n_edits, indel_pct, r, v)
        return bytes(r)[:n], bytes(v)[:m]

    def splitmix64_at(self, seed: int, k: int) -> int:
        return self.L.or_splitmix64_at(seed, k)


class Reference:
    """The reference's own src/c, compiled from /root/reference (oracle/_ref)."""

    def __init__(self, path: str = _REF_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        L = self.L = C.CDLL(path)
        u8p, sz = C.POINTER(C.c_uint8), C.c_size_t
        L.ref_encode_pair.restype = sz
        L.ref_encode_pair.argtypes = [C.c_int, u8p, sz, u8p, sz, sz, sz, sz, sz, C.POINTER(u8p)]
        L.ref_encode_pair_inplace.restype = sz
        L.ref_encode_pair_inplace.argtypes = [C.c_int, u8p, sz, u8p, sz, sz, sz, C.c_int,
                                              C.POINTER(u8p)]
        L.ref_free.argtypes = [C.c_void_p]

    def encode_inplace(self, algo: int, R: bytes, V: bytes, p: int = SEED_LEN,
                       q: int = TABLE_SIZE, policy: int = 0) -> bytes:
        """main.c encode --inplace [--policy localmin|constant]: an in-place delta."""
        out = C.POINTER(C.c_uint8)()
        n = self.L.ref_encode_pair_inplace(algo, _buf(R), len(R), _buf(V), len(V), p, q, policy,
                                           C.byref(out))
        res = C.string_at(out, n)
        self.L.ref_free(out)
        return res

    def encode(self, algo: int, R: bytes, V: bytes, p: int = SEED_LEN, q: int = TABLE_SIZE,
               buf_cap: int = BUF_CAP, max_table: int = MAX_TABLE) -> bytes:
        out = C.POINTER(C.c_uint8)()
        n = self.L.ref_encode_pair(algo, _buf(R), len(R), _buf(V), len(V), p, q, buf_cap,
                                   max_table, C.byref(out))
        res = C.string_at(out, n)
        self.L.ref_free(out)
        return res


def reference_available() -> bool:
    return os.path.exists(_REF_SO)

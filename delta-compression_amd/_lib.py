"""ctypes binding of libdeltagpu.so (include/delta_gpu.h).

Device buffers are passed as integer device addresses (e.g. a torch tensor's
``data_ptr()``) and streams as integer ``hipStream_t`` handles (e.g.
``torch.cuda.current_stream().cuda_stream``).  No torch type crosses the C ABI.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from dataclasses import dataclass
from typing import Iterable, List, Optional, Sequence, Tuple

HERE = os.path.dirname(os.path.abspath(__file__))
# DG_LIB_VARIANT=prof selects the profiling build (make prof); never a CPU path
_VARIANT = os.environ.get("DG_LIB_VARIANT", "")
LIB_PATH = os.path.join(HERE, "lib", "libdeltagpu%s.so" % ("_" + _VARIANT if _VARIANT else ""))

ALGO_GREEDY, ALGO_ONEPASS, ALGO_CORRECTING = 0, 1, 2
SEED_LEN = 16
TABLE_SIZE = 1048573
MAX_TABLE_SIZE = 1073741827
BUF_CAP = 256
OPT_VERBOSE, OPT_SPLAY, OPT_INPLACE, OPT_POLICY_CONSTANT = 0, 1, 2, 3
POLICIES = {"localmin": 0, "constant": 1}
CMD_COPY, CMD_ADD = 0, 1   # DG_CMD_COPY / DG_CMD_ADD

_ALGOS = {"greedy": ALGO_GREEDY, "onepass": ALGO_ONEPASS, "correcting": ALGO_CORRECTING}

STATUS = {
    0: "DG_OK", 1: "DG_ERR_INVALID_ARG", 2: "DG_ERR_UNSUPPORTED", 3: "DG_ERR_TOO_LARGE",
    4: "DG_ERR_NO_DEVICE", 5: "DG_ERR_HIP", 6: "DG_ERR_NOMEM", 7: "DG_ERR_CAPACITY",
    8: "DG_ERR_MALFORMED", 9: "DG_ERR_SRC_CRC", 10: "DG_ERR_DST_CRC", 11: "DG_ERR_TABLE_POOL", 12: "DG_ERR_INTERNAL",
}
LIMIT_TABLE_POOL_BYTES = 0
LIMIT_ONEPASS_MEMBERS = 1
MEMBERS_AUTO, MEMBERS_ON, MEMBERS_OFF = 0, 1, 2


class DeltaError(RuntimeError):
    def __init__(self, code: int, msg: str = ""):
        self.code = code
        super().__init__(f"{STATUS.get(code, code)}: {msg}" if msg else STATUS.get(code, str(code)))


class DiffOptions(C.Structure):
    """delta_diff_options_t (src/c/delta.h:248-257)."""
    _fields_ = [("p", C.c_size_t), ("q", C.c_size_t), ("buf_cap", C.c_size_t),
                ("max_table", C.c_size_t), ("flags", C.c_uint64)]

    @classmethod
    def make(cls, p: int = SEED_LEN, q: int = TABLE_SIZE, buf_cap: int = BUF_CAP,
             max_table: int = MAX_TABLE_SIZE, flags: int = 0) -> "DiffOptions":
        return cls(p, q, buf_cap, max_table, flags)


class Buffer(C.Structure):
    _fields_ = [("data", C.POINTER(C.c_uint8)), ("len", C.c_size_t)]


class Pair(C.Structure):
    _fields_ = [("r_off", C.c_uint64), ("r_len", C.c_uint64),
                ("v_off", C.c_uint64), ("v_len", C.c_uint64)]


class Span(C.Structure):
    _fields_ = [("off", C.c_uint64), ("len", C.c_uint64)]


class DecodeDesc(C.Structure):
    _fields_ = [("ref_off", C.c_uint64), ("ref_len", C.c_uint64),
                ("delta_off", C.c_uint64), ("delta_len", C.c_uint64),
                ("out_off", C.c_uint64), ("out_cap", C.c_uint64)]


class InplaceStats(C.Structure):
    _fields_ = [("already_inplace", C.c_int), ("num_copies", C.c_uint64), ("num_adds", C.c_uint64),
                ("copy_bytes", C.c_uint64), ("add_bytes", C.c_uint64)]


class DeltaInfo(C.Structure):
    _fields_ = [("inplace", C.c_int), ("version_size", C.c_uint64),
                ("src_crc", C.c_uint8 * 8), ("dst_crc", C.c_uint8 * 8),
                ("num_commands", C.c_uint64), ("num_copies", C.c_uint64),
                ("num_adds", C.c_uint64), ("copy_bytes", C.c_uint64),
                ("add_bytes", C.c_uint64)]


class PlacedCommandC(C.Structure):   # dg_placed_command_t
    _fields_ = [("tag", C.c_uint32), ("src", C.c_uint64), ("dst", C.c_uint64), ("length", C.c_uint64),
                ("data", C.POINTER(C.c_uint8))]


class Commands(C.Structure):         # dg_commands_t
    _fields_ = [("data", C.POINTER(PlacedCommandC)), ("len", C.c_size_t), ("storage", C.c_void_p)]


def _share_torch_runtime() -> None:
    """One HIP runtime per process.

    PyTorch-ROCm ships its own libamdhip64/libhsa-runtime64.  If libdeltagpu.so
    were loaded first it would bind /opt/rocm's runtime and torch would then
    load a second one, which cannot open the device again ("No HIP GPUs are
    available").  Importing torch first makes the dynamic linker satisfy our
    libamdhip64.so.7 dependency with torch's already-loaded copy, so device
    pointers and streams are shared by construction.
    """
    try:
        import torch  # noqa: F401
    except Exception:  # torch absent: /opt/rocm's runtime is used
        pass


def _load() -> C.CDLL:
    _share_torch_runtime()
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `make -C delta-compression_amd` "
            "(or __graft_entry__.build()); there is no CPU fallback")
    L = C.CDLL(LIB_PATH)
    vp, u8p, sz, u32, u64, i32 = C.c_void_p, C.POINTER(C.c_uint8), C.c_size_t, C.c_uint32, C.c_uint64, C.c_int32
    sig = {
        "dg_abi_version": (C.c_int, []),
        "dg_diff_options_default": (None, [C.POINTER(DiffOptions)]),
        "dg_buffer_free": (None, [C.POINTER(Buffer)]),
        "dg_context_create": (C.c_int, [C.c_int, C.POINTER(vp)]),
        "dg_context_destroy": (None, [vp]),
        "dg_context_stream": (vp, [vp]),
        "dg_context_set_limit": (C.c_int, [vp, C.c_int, u64]),
        "dg_status_string": (C.c_char_p, [C.c_int]),
        "dg_last_error": (C.c_char_p, [vp]),
        "dg_encode_plan_create": (C.c_int, [vp, C.c_int, C.POINTER(Pair), u32, C.POINTER(DiffOptions), C.POINTER(vp)]),
        "dg_encode_plan_output_bound": (u64, [vp]),
        "dg_encode_plan_num_pairs": (u32, [vp]),
        "dg_encode_plan_flags": (u32, [vp]),
        "dg_encode_plan_run_modes": (C.c_int, [vp, C.POINTER(u64), C.POINTER(u64)]),
        "dg_encode_plan_table_size": (u64, [vp, u32]),
        "dg_encode_plan_run": (C.c_int, [vp, vp, vp, vp, u64, vp, vp, vp]),
        "dg_encode_plan_set_timing": (C.c_int, [vp, C.c_int]),
        "dg_encode_plan_set_timing_mode": (C.c_int, [vp, C.c_int]),
        "dg_encode_plan_set_timing_every": (C.c_int, [vp, C.c_int]),
        "dg_encode_plan_stage_times": (C.c_int, [vp, C.POINTER(C.c_float), C.POINTER(C.c_char_p), C.c_int]),
        "dg_encode_plan_copy_counts_device": (vp, [vp]),
        "dg_encode_plan_destroy": (None, [vp]),
        "dg_encode": (C.c_int, [vp, C.c_int, u8p, sz, u8p, sz, C.POINTER(DiffOptions), C.POINTER(Buffer)]),
        "dg_encode_batch": (C.c_int, [vp, C.c_int, C.POINTER(u8p), C.POINTER(sz), C.POINTER(u8p),
                                      C.POINTER(sz), u32, C.POINTER(DiffOptions), C.POINTER(Buffer),
                                      C.POINTER(i32)]),
        "dg_encode_pipelined": (C.c_int, [vp, C.c_int, vp, vp, C.POINTER(Pair), u32, C.POINTER(DiffOptions), u64,
                                          vp, u64, C.POINTER(u64), C.POINTER(i32)]),
        "dg_encode_pipelined_multi": (C.c_int, [C.POINTER(vp), u32, C.c_int, vp, vp, C.POINTER(Pair), u32,
                                                C.POINTER(DiffOptions), u64, vp, u64, C.POINTER(u64), C.POINTER(i32)]),
        "dg_host_alloc": (C.c_int, [vp, u64, C.POINTER(vp)]),
        "dg_host_free": (None, [vp]),
        "dg_crc64_xz": (C.c_int, [vp, u8p, sz, C.c_uint8 * 8]),
        "dg_crc64_xz_batch_device": (C.c_int, [vp, vp, C.POINTER(Span), u32, vp, vp]),
        "dg_decode": (C.c_int, [vp, u8p, sz, u8p, sz, C.c_int, C.POINTER(Buffer)]),
        "dg_decode_batch_device": (C.c_int, [vp, vp, vp, C.POINTER(DecodeDesc), u32, C.c_int, vp, vp, vp, vp]),
        "dg_decode_plan_create": (C.c_int, [vp, C.POINTER(DecodeDesc), u32, C.c_int, C.POINTER(vp)]),
        "dg_decode_plan_run": (C.c_int, [vp, vp, vp, vp, vp, vp, vp]),
        "dg_decode_plan_set_timing": (C.c_int, [vp, C.c_int]),
        "dg_decode_plan_set_timing_every": (C.c_int, [vp, C.c_int]),
        "dg_decode_plan_stage_times": (C.c_int, [vp, C.POINTER(C.c_float), C.POINTER(C.c_char_p), C.c_int]),
        "dg_decode_plan_destroy": (None, [vp]),
        "dg_delta_info": (C.c_int, [u8p, sz, C.POINTER(DeltaInfo)]),
        "dg_diff": (C.c_int, [vp, C.c_int, u8p, sz, u8p, sz, C.POINTER(DiffOptions), C.POINTER(Commands)]),
        "dg_delta_decode": (C.c_int, [u8p, sz, C.POINTER(Commands), C.POINTER(DeltaInfo)]),
        "dg_encode_commands": (C.c_int, [C.POINTER(PlacedCommandC), sz, C.c_int, u64, C.c_uint8 * 8,
                                         C.c_uint8 * 8, C.POINTER(Buffer)]),
        "dg_commands_free": (None, [C.POINTER(Commands)]),
        "dg_make_inplace": (C.c_int, [u8p, sz, u8p, sz, C.c_int, C.POINTER(Buffer), C.POINTER(InplaceStats)]),
        "dg_synth_edit_pairs_device": (C.c_int, [vp, vp, vp, u32, u64, u64, u64, vp]),
        "dg_synth_shift_pairs_device": (C.c_int, [vp, u64, u32, u64, u64, u32, C.POINTER(Pair),
                                                  C.POINTER(u64), C.POINTER(u64), vp, vp, vp]),
        "dg_synth_transpose_pairs_device": (C.c_int, [vp, u64, u32, u64, u32, C.POINTER(Pair),
                                                      C.POINTER(u64), C.POINTER(u64), vp, vp, vp]),
    }
    for name, (res, args) in sig.items():
        try:
            fn = getattr(L, name)
        except AttributeError:
            if os.environ.get("DG_LIB_VARIANT"):   # an older A/B baseline build
                continue
            raise
        fn.restype = res
        fn.argtypes = args
    return L


lib = _load()


def _set_every(fn, plan, every):
    if fn is not None:
        plan.ctx.check(fn(plan.handle, int(every)), "timing stride")
    elif every != 1:   # (older A/B variant builds lack it)
        raise RuntimeError("this library build records events on every run only")


def status_string(code: int) -> str:
    return lib.dg_status_string(code).decode()


def _u8(b: bytes):
    return C.cast(C.c_char_p(b), C.POINTER(C.c_uint8)) if b else None


def _opts(p=SEED_LEN, q=TABLE_SIZE, buf_cap=BUF_CAP, max_table=MAX_TABLE_SIZE, flags=0,
          verbose=False, splay=False, inplace=False, policy="localmin") -> DiffOptions:
    f = flags | (verbose << OPT_VERBOSE) | (splay << OPT_SPLAY) | (inplace << OPT_INPLACE)
    f |= POLICIES[policy] << OPT_POLICY_CONSTANT
    return DiffOptions.make(p, q, buf_cap, max_table, f)


def _algo(a) -> int:
    if isinstance(a, str):
        if a not in _ALGOS:
            raise ValueError(f"Unknown algorithm: {a}")
        return _ALGOS[a]
    return int(a)


class Context:
    """A HIP device + stream + constant tables (dg_context_t)."""

    def __init__(self, device: int = -1):
        h = C.c_void_p()
        rc = lib.dg_context_create(device, C.byref(h))
        if rc:
            raise DeltaError(rc, "dg_context_create")
        self.handle = h

    def close(self):
        if self.handle:
            lib.dg_context_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self) -> int:
        return lib.dg_context_stream(self.handle) or 0

    def set_limit(self, limit: int, value: int):
        """dg_context_set_limit (e.g. LIMIT_TABLE_POOL_BYTES; 0 = automatic)."""
        self.check(lib.dg_context_set_limit(self.handle, int(limit), int(value)), "set_limit")

    def check(self, rc: int, what: str = ""):
        if rc:
            raise DeltaError(rc, f"{what}: {lib.dg_last_error(self.handle).decode()}")


_default_ctx: Optional[Context] = None
_ctx_lock = threading.Lock()


def default_context() -> Context:
    global _default_ctx
    with _ctx_lock:
        if _default_ctx is None:
            _default_ctx = Context(-1)
        return _default_ctx


class EncodePlan:
    """Device-resident batch (dg_encode_plan_t): fixed pair geometry + options.

    ``pairs`` is a sequence of (r_off, r_len, v_off, v_len) into two device
    arenas.  ``run`` takes device addresses and an optional stream handle.
    """

    def __init__(self, ctx: Context, algorithm, pairs: Sequence[Tuple[int, int, int, int]],
                 **opt_kw):
        self.ctx = ctx
        n = len(pairs)
        arr = (Pair * max(n, 1))(*[Pair(*p) for p in pairs])
        o = _opts(**opt_kw)
        h = C.c_void_p()
        ctx.check(lib.dg_encode_plan_create(ctx.handle, _algo(algorithm), arr, n, C.byref(o),
                                            C.byref(h)), "dg_encode_plan_create")
        self.handle = h
        self.n = n

    @property
    def output_bound(self) -> int:
        return lib.dg_encode_plan_output_bound(self.handle)

    @property
    def members(self) -> bool:
        """True when onepass runs through verified diagonal members."""
        fn = getattr(lib, "dg_encode_plan_flags", None)   # (absent from older A/B baselines)
        return bool(fn(self.handle) & 1) if fn else False

    @property
    def run_modes(self) -> tuple:
        """(runs in member mode, runs as a plain plan) so far: automatic member
        mode runs a batch whose every pair it routed to the plain chain as a
        plain plan between member-mode probes (dg_encode_plan_run_modes)."""
        fn = getattr(lib, "dg_encode_plan_run_modes", None)   # (absent from older A/B baselines)
        if not fn:
            return (0, 0)
        m, p = C.c_uint64(), C.c_uint64()
        self.ctx.check(fn(self.handle, C.byref(m), C.byref(p)), "dg_encode_plan_run_modes")
        return (m.value, p.value)

    def table_size(self, i: int) -> int:
        return lib.dg_encode_plan_table_size(self.handle, i)

    def set_timing(self, slots: int = 1, dominant_only: bool = False, every: int = 1):
        """Record per-stage events for the next runs (ring of `slots` sets);
        dominant_only: only the events around the dominant kernel(s);
        every: only every `every`-th run records them."""
        mode = getattr(lib, "dg_encode_plan_set_timing_mode", None)   # (older A/B variant builds lack it)
        if mode is not None:
            self.ctx.check(mode(self.handle, 1 if dominant_only else 0), "timing mode")
        _set_every(getattr(lib, "dg_encode_plan_set_timing_every", None), self, every)
        self.ctx.check(lib.dg_encode_plan_set_timing(self.handle, int(slots)), "set_timing")

    def stage_times(self):
        ms = (C.c_float * 8)()
        names = (C.c_char_p * 8)()
        k = lib.dg_encode_plan_stage_times(self.handle, ms, names, 8)
        return {names[i].decode(): ms[i] for i in range(k)}

    def copy_counts_ptr(self) -> int:
        return lib.dg_encode_plan_copy_counts_device(self.handle) or 0

    def run(self, d_ref: int, d_ver: int, d_out: int, out_cap: int, d_offsets: int,
            d_status: int, stream: int = 0):
        self.ctx.check(lib.dg_encode_plan_run(self.handle, d_ref, d_ver, d_out, out_cap, d_offsets,
                                              d_status, stream or None), "dg_encode_plan_run")

    def close(self):
        if getattr(self, "handle", None):
            lib.dg_encode_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DecodePlan:
    """dg_decode_plan_t: batched device decode + CRC verify (C5)."""

    def __init__(self, ctx: Context, descs: Sequence[Tuple[int, int, int, int, int, int]],
                 ignore_hash: bool = False):
        self.ctx = ctx
        n = len(descs)
        arr = (DecodeDesc * max(n, 1))(*[DecodeDesc(*d) for d in descs])
        h = C.c_void_p()
        ctx.check(lib.dg_decode_plan_create(ctx.handle, arr, n, int(ignore_hash), C.byref(h)),
                  "dg_decode_plan_create")
        self.handle = h
        self.n = n

    def run(self, d_ref: int, d_delta: int, d_out: int, d_out_len: int, d_status: int,
            stream: int = 0):
        self.ctx.check(lib.dg_decode_plan_run(self.handle, d_ref, d_delta, d_out, d_out_len, d_status,
                                              stream or None), "dg_decode_plan_run")

    def set_timing(self, slots: int = 1, every: int = 1):
        """Events around the kernel on every `every`-th run (ring of `slots`)."""
        _set_every(getattr(lib, "dg_decode_plan_set_timing_every", None), self, every)
        self.ctx.check(lib.dg_decode_plan_set_timing(self.handle, int(slots)), "set_timing")

    def stage_times(self):
        ms = (C.c_float * 8)()
        names = (C.c_char_p * 8)()
        k = lib.dg_decode_plan_stage_times(self.handle, ms, names, 8)
        return {names[i].decode(): ms[i] for i in range(k)}

    def close(self):
        if self.handle:
            lib.dg_decode_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def encode(R: bytes, V: bytes, algorithm="onepass", p: int = SEED_LEN, q: int = TABLE_SIZE,
           buf_cap: int = BUF_CAP, max_table: int = MAX_TABLE_SIZE, splay: bool = False,
           inplace: bool = False, policy: str = "localmin",
           ctx: Optional[Context] = None) -> bytes:
    """One pair, host bytes in, DLT\\x03 bytes out (src/c/main.c:257-292)."""
    ctx = ctx or default_context()
    out = Buffer()
    o = _opts(p, q, buf_cap, max_table, splay=splay, inplace=inplace, policy=policy)
    rc = lib.dg_encode(ctx.handle, _algo(algorithm), _u8(R), len(R), _u8(V), len(V), C.byref(o),
                       C.byref(out))
    ctx.check(rc, "dg_encode")
    res = C.string_at(out.data, out.len)
    lib.dg_buffer_free(C.byref(out))
    return res


def encode_batch(pairs: Sequence[Tuple[bytes, bytes]], algorithm="onepass", p: int = SEED_LEN,
                 q: int = TABLE_SIZE, buf_cap: int = BUF_CAP, max_table: int = MAX_TABLE_SIZE,
                 ctx: Optional[Context] = None) -> List[bytes]:
    """Many pairs through the batched device path (host buffers in and out)."""
    ctx = ctx or default_context()
    n = len(pairs)
    if n == 0:
        return []
    keep = [(bytes(r), bytes(v)) for r, v in pairs]
    rp = (C.POINTER(C.c_uint8) * n)(*[_u8(r) for r, _ in keep])
    vp = (C.POINTER(C.c_uint8) * n)(*[_u8(v) for _, v in keep])
    rl = (C.c_size_t * n)(*[len(r) for r, _ in keep])
    vl = (C.c_size_t * n)(*[len(v) for _, v in keep])
    outs = (Buffer * n)()
    st = (C.c_int32 * n)()
    o = _opts(p, q, buf_cap, max_table)
    ctx.check(lib.dg_encode_batch(ctx.handle, _algo(algorithm), rp, rl, vp, vl, n, C.byref(o), outs,
                                  st), "dg_encode_batch")
    res = []
    for i in range(n):
        if st[i]:
            raise DeltaError(st[i], f"pair {i}")
        res.append(C.string_at(outs[i].data, outs[i].len))
        lib.dg_buffer_free(C.byref(outs[i]))
    return res


def encode_pipelined(pairs: Sequence[Tuple[bytes, bytes]], algorithm="onepass", p: int = SEED_LEN,
                     q: int = TABLE_SIZE, buf_cap: int = BUF_CAP, max_table: int = MAX_TABLE_SIZE,
                     chunk_bytes: int = 0, pinned: bool = False, align: int = 16, out_cap: Optional[int] = None,
                     ctx: Optional[Context] = None, ctxs: Optional[Sequence[Context]] = None) -> List[bytes]:
    """Many pairs host-to-host through dg_encode_pipelined (chunked, two chunks in
    flight).  The pairs are laid out in host arenas `align` bytes apart, pinned
    (dg_host_alloc) or pageable (bytearray).  ctxs: one context per device,
    through dg_encode_pipelined_multi (byte-balanced pair ranges, one host
    thread per device, deltas packed in pair order)."""
    ctx = ctx or (ctxs[0] if ctxs else default_context())
    n = len(pairs)
    if n == 0:
        return []
    lay, rt, vt = [], 0, 0
    for r, v in pairs:   # each pair at the next multiple of `align` (1: packed, unaligned)
        ro, vo = (rt + align - 1) // align * align, (vt + align - 1) // align * align
        lay.append((ro, len(r), vo, len(v)))
        rt, vt = ro + len(r), vo + len(v)
    cap = out_cap if out_cap is not None else sum(len(v) for _, v in pairs) + 64 * n + 64
    bufs = []

    def host(nbytes):
        if pinned:
            h = C.c_void_p()
            ctx.check(lib.dg_host_alloc(ctx.handle, max(nbytes, 1), C.byref(h)), "dg_host_alloc")
            bufs.append(h)
            return h.value
        b = (C.c_uint8 * max(nbytes, 1))()
        bufs.append(b)
        return C.addressof(b)

    try:
        hr, hv, ho = host(rt), host(vt), host(cap)
        for (r, v), (ro, _, vo, _) in zip(pairs, lay):
            C.memmove(hr + ro, bytes(r), len(r))
            C.memmove(hv + vo, bytes(v), len(v))
        pa = (Pair * n)(*[Pair(*x) for x in lay])
        offs = (C.c_uint64 * (n + 1))()
        st = (C.c_int32 * n)()
        o = _opts(p, q, buf_cap, max_table)
        if ctxs:
            hs = (C.c_void_p * len(ctxs))(*[c.handle for c in ctxs])
            ctx.check(lib.dg_encode_pipelined_multi(hs, len(ctxs), _algo(algorithm), hr, hv, pa, n, C.byref(o),
                                                    chunk_bytes, ho, cap, offs, st), "dg_encode_pipelined_multi")
        else:
            ctx.check(lib.dg_encode_pipelined(ctx.handle, _algo(algorithm), hr, hv, pa, n, C.byref(o), chunk_bytes,
                                              ho, cap, offs, st), "dg_encode_pipelined")
        res = []
        for i in range(n):
            if st[i]:
                raise DeltaError(st[i], f"pair {i}")
            res.append(C.string_at(ho + offs[i], offs[i + 1] - offs[i]))
        return res
    finally:
        if pinned:
            for h in bufs:
                lib.dg_host_free(h)


def make_inplace(R: bytes, delta: bytes, policy: str = "localmin", stats: bool = False):
    """main.c `inplace` (:427-480): standard delta -> in-place delta, host only."""
    out = Buffer()
    st = InplaceStats()
    rc = lib.dg_make_inplace(_u8(R), len(R), _u8(delta), len(delta), POLICIES[policy], C.byref(out),
                             C.byref(st))
    if rc:
        raise DeltaError(rc, "dg_make_inplace")
    res = C.string_at(out.data, out.len) if out.len else b""
    lib.dg_buffer_free(C.byref(out))
    if stats:
        return res, {k: getattr(st, k) for k, _ in InplaceStats._fields_}
    return res


def crc64_xz(data: bytes, ctx: Optional[Context] = None) -> bytes:
    """CRC-64/XZ, 8 bytes big-endian (src/c/delta.h:294-322), on the GPU."""
    ctx = ctx or default_context()
    out = (C.c_uint8 * 8)()
    ctx.check(lib.dg_crc64_xz(ctx.handle, _u8(data), len(data), out), "dg_crc64_xz")
    return bytes(out)


def decode(R: bytes, delta: bytes, ignore_hash: bool = False,
           ctx: Optional[Context] = None) -> bytes:
    """Apply a delta to R on the GPU (src/c/main.c:323-400)."""
    ctx = ctx or default_context()
    out = Buffer()
    rc = lib.dg_decode(ctx.handle, _u8(R), len(R), _u8(delta), len(delta), int(ignore_hash),
                       C.byref(out))
    res = C.string_at(out.data, out.len) if out.len else b""
    lib.dg_buffer_free(C.byref(out))
    ctx.check(rc, "dg_decode")
    return res


def info(delta: bytes) -> dict:
    """Header and command summary (src/c/main.c:402-425)."""
    d = DeltaInfo()
    rc = lib.dg_delta_info(_u8(delta), len(delta), C.byref(d))
    if rc:
        raise DeltaError(rc, "dg_delta_info")
    return {
        "inplace": bool(d.inplace), "version_size": d.version_size,
        "src_crc": bytes(d.src_crc), "dst_crc": bytes(d.dst_crc),
        "num_commands": d.num_commands, "num_copies": d.num_copies, "num_adds": d.num_adds,
        "copy_bytes": d.copy_bytes, "add_bytes": d.add_bytes,
    }


# ── command lists (src/python/delta.py:44-96, 854-1000; delta.h:94-137) ──────

@dataclass
class CopyCmd:
    """Copy R[offset : offset+length] to the output (delta.py:44-51)."""
    offset: int
    length: int


@dataclass
class AddCmd:
    """Append literal bytes (delta.py:54-62)."""
    data: bytes


@dataclass
class PlacedCopy:
    """COPY with explicit source and destination (delta.py:72-80)."""
    src: int
    dst: int
    length: int


@dataclass
class PlacedAdd:
    """ADD at an explicit destination (delta.py:83-92)."""
    dst: int
    data: bytes


def _placed_list(cl: Commands) -> list:
    out = []
    for i in range(cl.len):
        c = cl.data[i]
        if c.tag == CMD_COPY:
            out.append(PlacedCopy(c.src, c.dst, c.length))
        else:
            out.append(PlacedAdd(c.dst, C.string_at(c.data, c.length) if c.length else b""))
    return out


def diff(R: bytes, V: bytes, algorithm="onepass", p: int = SEED_LEN, q: int = TABLE_SIZE,
         buf_cap: int = BUF_CAP, max_table: int = MAX_TABLE_SIZE, verbose: bool = False,
         ctx: Optional[Context] = None) -> list:
    """delta_diff / diff_onepass / diff_correcting (delta.py:376, 576): the
    algorithm's commands (CopyCmd / AddCmd), computed by the GPU encoder
    (dg_diff)."""
    return unplace_commands(diff_placed(R, V, algorithm, p, q, buf_cap, max_table, verbose, ctx))


def diff_placed(R: bytes, V: bytes, algorithm="onepass", p: int = SEED_LEN, q: int = TABLE_SIZE,
                buf_cap: int = BUF_CAP, max_table: int = MAX_TABLE_SIZE, verbose: bool = False,
                ctx: Optional[Context] = None) -> list:
    """place_commands(diff(...)) in one call (dg_diff returns the placed form)."""
    ctx = ctx or default_context()
    cl = Commands()
    o = _opts(p, q, buf_cap, max_table, verbose=verbose)
    ctx.check(lib.dg_diff(ctx.handle, _algo(algorithm), _u8(R), len(R), _u8(V), len(V), C.byref(o),
                          C.byref(cl)), "dg_diff")
    try:
        return _placed_list(cl)
    finally:
        lib.dg_commands_free(C.byref(cl))


def diff_onepass(R: bytes, V: bytes, p: int = SEED_LEN, q: int = TABLE_SIZE, **kw) -> list:
    return diff(R, V, "onepass", p=p, q=q, **kw)


def diff_correcting(R: bytes, V: bytes, p: int = SEED_LEN, q: int = TABLE_SIZE,
                    buf_cap: int = BUF_CAP, **kw) -> list:
    return diff(R, V, "correcting", p=p, q=q, buf_cap=buf_cap, **kw)


def output_size(commands: list) -> int:
    """delta.py:848-851."""
    return sum(c.length if isinstance(c, CopyCmd) else len(c.data) for c in commands)


def place_commands(commands: list) -> list:
    """Sequential destinations (delta.py:854-865, apply.c:136-164)."""
    out, dst = [], 0
    for c in commands:
        if isinstance(c, CopyCmd):
            out.append(PlacedCopy(c.offset, dst, c.length))
            dst += c.length
        else:
            out.append(PlacedAdd(dst, bytes(c.data)))
            dst += len(c.data)
    return out


def unplace_commands(placed: list) -> list:
    """Placed -> algorithm commands in destination order, stable
    (delta.py:868-895, apply.c:168-225)."""
    order = sorted(range(len(placed)), key=lambda i: placed[i].dst)
    return [CopyCmd(placed[i].src, placed[i].length) if isinstance(placed[i], PlacedCopy)
            else AddCmd(placed[i].data) for i in order]


def encode_delta(commands: list, *, inplace: bool = False, version_size: int, src_crc: bytes,
                 dst_crc: bytes) -> bytes:
    """Placed commands -> DLT\\x03 bytes (delta.py:939-964) via dg_encode_commands."""
    if len(src_crc) != 8 or len(dst_crc) != 8:
        raise ValueError("src_crc and dst_crc must be 8 bytes")
    n = len(commands)
    arr = (PlacedCommandC * max(n, 1))()
    keep = []
    for i, c in enumerate(commands):
        if isinstance(c, PlacedCopy):
            arr[i] = PlacedCommandC(CMD_COPY, c.src, c.dst, c.length, None)
        else:
            b = bytes(c.data)
            keep.append(b)
            arr[i] = PlacedCommandC(CMD_ADD, 0, c.dst, len(b), _u8(b))
    out = Buffer()
    rc = lib.dg_encode_commands(arr, n, int(inplace), version_size, (C.c_uint8 * 8)(*src_crc),
                                (C.c_uint8 * 8)(*dst_crc), C.byref(out))
    if rc:
        raise DeltaError(rc, "dg_encode_commands")
    try:
        return C.string_at(out.data, out.len)
    finally:
        lib.dg_buffer_free(C.byref(out))


def decode_delta(data: bytes):
    """delta.py:967-999's name and return value (commands, inplace,
    version_size, src_crc, dst_crc), via dg_delta_decode.  Malformed input
    follows the C decoder (encoding.c:111-178), not delta.py: an unknown
    command type or a COPY/ADD cut short by the buffer end raises
    DeltaError (code 8) where delta.py skips unknown types and returns
    truncated ADD data.  tests/test_format_cpu.py::test_decode_errors pins
    this choice."""
    cl, hdr = Commands(), DeltaInfo()
    rc = lib.dg_delta_decode(_u8(data), len(data), C.byref(cl), C.byref(hdr))
    if rc:
        raise DeltaError(rc, "dg_delta_decode")
    try:
        return (_placed_list(cl), bool(hdr.inplace), hdr.version_size, bytes(hdr.src_crc),
                bytes(hdr.dst_crc))
    finally:
        lib.dg_commands_free(C.byref(cl))

"""fri_amd — Python host mirror of the reference FRI-commit interface over
``libfri_amd.so`` (C ABI: include/fri_amd.h).

Mirrors the reference crate's surface for this path (same names, argument
meaning, error behaviour):

* ``Channel``            — src/channel/channel.rs (send / receive_random_field_element /
                           receive_random_int / proof / proof_size)
* ``MerkleTree``         — src/merkle/mod.rs (``MerkleTree(values).root() -> hex str``)
* ``fri_commit``         — src/fri/fri_commit.rs:72-122, returns ``FRIProof``
* ``lde`` / ``interpolate`` / ``evaluate`` / ``batch_inverse`` / ``fold`` — the
  polynomial / field kernels (src/polynomial/ops.rs, interpolation.rs,
  src/fields/element.rs, src/fri/fri_commit.rs:53-65).

Every compute call goes through the HIP library; there is no CPU fallback.
If the library or a gfx950 GPU is missing the calls raise ``FriError``.
Where the reference panics, these raise ``FriError`` as well.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

P = 3221225473
GENERATOR = 5
MAX_ROUNDS = 32

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.normpath(os.path.join(_HERE, "..", "lib", os.environ.get("FRI_AMD_LIB", "libfri_amd.so")))
HEADER_PATH = os.path.normpath(os.path.join(_HERE, "..", "..", "include", "fri_amd.h"))

FRI_OK, FRI_EINVAL, FRI_ENOMEM, FRI_EHIP, FRI_ENODEV, FRI_ERCCL, FRI_ESTATE, FRI_EDEGREE = range(8)
FLAG_FORCE_BETAS = 1
FLAG_NO_GRAPH = 2
FLAG_RANK_INPUTS = 4      # FRI_FLAG_RANK_INPUTS (fri_amd.h): team commit from the ranks' resident inputs
MAX_INFLIGHT = 4          # FRI_MAX_INFLIGHT (fri_amd.h): pipelined commits pending per context
DEFAULT_LANES = 3         # FRI_DEFAULT_LANES (fri_amd.h): commit lanes of a context


class FriError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"fri_amd error {code}: {msg}")
        self.code = code


class ChannelState(ctypes.Structure):
    _fields_ = [("digest", ctypes.c_uint8 * 32), ("has_state", ctypes.c_uint32)]


class CommitResult(ctypes.Structure):
    _fields_ = [("n_layers", ctypes.c_uint32), ("n_rounds", ctypes.c_uint32), ("log_n", ctypes.c_uint32),
                ("final_value", ctypes.c_uint32), ("final_degree", ctypes.c_int32),
                ("reserved", ctypes.c_uint32),
                ("roots", (ctypes.c_uint8 * 32) * (MAX_ROUNDS + 1)),
                ("betas", ctypes.c_uint32 * MAX_ROUNDS),
                ("channel_out", ChannelState)]


class Collectives(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p),
                ("allgather", ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_size_t)),
                ("alltoall", ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_size_t)),
                ("sendrecv", ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_size_t, ctypes.c_int))]


class TransportOp(ctypes.Structure):
    """fri_transport_op: one entry of fri_debug_transport_log."""
    _fields_ = [("chan", ctypes.c_uint32), ("op", ctypes.c_uint32), ("peer", ctypes.c_int32),
                ("reserved", ctypes.c_uint32), ("bytes", ctypes.c_uint64)]


TRANSPORT_OPS = {1: "allgather", 2: "alltoall", 3: "sendrecv"}
TRANSPORTS = ("none", "rccl", "host", "loopback", "peer")     # FRI_TRANSPORT_* (fri_amd.h)

_lib = None


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libfri_amd.so; raises FriError if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise FriError(FRI_ENODEV, f"{path} missing: build it with `make -C stark-prover_amd`")
    lib = ctypes.CDLL(path)
    u32, sz, i32 = ctypes.c_uint32, ctypes.c_size_t, ctypes.c_int
    pu32 = ctypes.POINTER(ctypes.c_uint32)
    vp = ctypes.c_void_p
    sig = {
        "fri_ctx_create": (i32, [i32, u32, ctypes.POINTER(vp)]),
        "fri_ctx_create_multi": (i32, [ctypes.POINTER(i32), u32, u32, i32, ctypes.POINTER(vp)]),
        "fri_debug_team_rank": (i32, [vp, u32, ctypes.POINTER(vp)]),
        "fri_debug_team_inject_failure": (i32, [vp, u32, ctypes.c_int64]),
        "fri_ctx_destroy": (i32, [vp]),
        "fri_last_error": (ctypes.c_char_p, [vp]),
        "fri_version": (ctypes.c_char_p, []),
        "fri_batch_inverse": (i32, [vp, pu32, pu32, sz]),
        "fri_lde": (i32, [vp, pu32, sz, u32, u32, pu32]),
        "fri_interpolate": (i32, [vp, pu32, u32, u32, pu32, ctypes.POINTER(sz)]),
        "fri_interpolate_points": (i32, [vp, pu32, pu32, sz, pu32, ctypes.POINTER(sz)]),
        "fri_evaluate": (i32, [vp, pu32, sz, pu32, sz, pu32]),
        "fri_fold": (i32, [vp, pu32, u32, u32, u32, pu32]),
        "fri_merkle_root": (i32, [vp, pu32, sz, ctypes.c_char_p]),
        "fri_commit": (i32, [vp, pu32, sz, u32, u32, ctypes.POINTER(ChannelState), u32, pu32,
                             ctypes.POINTER(CommitResult)]),
        "fri_commit_device": (i32, [vp, vp, sz, u32, u32, ctypes.POINTER(ChannelState), u32, pu32,
                                    ctypes.POINTER(CommitResult)]),
        "fri_commit_device_async": (i32, [vp, vp, sz, u32, u32, ctypes.POINTER(ChannelState), u32, pu32,
                                          ctypes.POINTER(ctypes.c_uint64)]),
        "fri_commit_wait": (i32, [vp, ctypes.c_uint64, ctypes.POINTER(CommitResult)]),
        "fri_commit_async": (i32, [vp, pu32, sz, u32, u32, ctypes.POINTER(ChannelState), u32, pu32,
                                   ctypes.POINTER(ctypes.c_uint64)]),
        "fri_ctx_input_buffer": (i32, [vp, sz, ctypes.POINTER(vp)]),
        "fri_ctx_input_upload": (i32, [vp, pu32, sz]),
        "fri_ctx_create_default": (i32, [u32, ctypes.POINTER(vp), ctypes.POINTER(u32)]),
        "fri_debug_team_force_copy": (i32, [vp, i32]),
        "fri_commit_info": (i32, [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(u32), ctypes.POINTER(u32)]),
        "fri_layer_copy": (i32, [vp, u32, pu32, sz]),
        "fri_tree_level_copy": (i32, [vp, u32, u32, ctypes.c_char_p, sz]),
        "fri_auth_path": (i32, [vp, u32, ctypes.c_uint64, pu32, ctypes.c_char_p, ctypes.POINTER(u32)]),
        "fri_trace_commit": (i32, [vp, pu32, u32, u32, u32, ctypes.c_char_p, pu32, ctypes.POINTER(sz), pu32]),
        "fri_decommit_query": (i32, [vp, ctypes.c_uint64, pu32, sz, ctypes.c_char_p, sz, ctypes.POINTER(sz)]),
        "fri_fibsq_composition_commit": (i32, [vp, u32, u32, u32, u32, pu32, ctypes.POINTER(ChannelState), u32,
                                               ctypes.POINTER(CommitResult)]),
        "fri_fibsq_trace": (i32, [u32, u32, pu32]),
        "fri_trace_decommit": (i32, [vp, ctypes.c_uint64, ctypes.c_uint64, u32, pu32, ctypes.c_char_p, sz]),
        "fri_set_profiling": (i32, [vp, i32]),
        "fri_get_profile": (i32, [vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                                  ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
        "fri_reset_profile": (i32, [vp]),
        "fri_debug_inject_stall": (i32, [vp, i32]),
        "fri_debug_attach_loopback": (i32, [vp, i32, i32]),
        "fri_debug_plan_layout": (i32, [sz, u32, u32, u32, ctypes.POINTER(ctypes.c_uint64), sz]),
        "fri_ctx_device_bytes": (i32, [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
        "fri_debug_set_device_cap": (i32, [vp, ctypes.c_uint64]),
        "fri_debug_stamps": (i32, [vp, ctypes.POINTER(ctypes.c_uint64), sz]),
        "fri_dist_unique_id": (i32, [ctypes.c_char_p]),
        "fri_dist_attach_rccl": (i32, [vp, i32, i32, ctypes.c_char_p]),
        "fri_dist_attach_host": (i32, [vp, i32, i32, ctypes.POINTER(Collectives)]),
        "fri_dist_detach": (i32, [vp]),
        "fri_dist_info": (i32, [vp, ctypes.POINTER(i32), ctypes.POINTER(i32), ctypes.POINTER(i32)]),
        "fri_dist_selftest": (i32, [vp, sz]),
        "fri_commit_sharded": (i32, [vp, pu32, sz, u32, u32, ctypes.POINTER(ChannelState), u32, pu32,
                                     ctypes.POINTER(CommitResult)]),
        "fri_commit_sharded_device": (i32, [vp, vp, sz, u32, u32, ctypes.POINTER(ChannelState), u32, pu32,
                                            ctypes.POINTER(CommitResult)]),
        "fri_decommit_query_sharded": (i32, [vp, ctypes.c_uint64, pu32, sz, ctypes.c_char_p, sz,
                                             ctypes.POINTER(sz)]),
        "fri_debug_loopback_degrees": (i32, [vp, ctypes.POINTER(ctypes.c_int32), u32]),
        "fri_ctx_set_lanes": (i32, [vp, u32]),
        "fri_debug_ticket_lane": (i32, [vp, ctypes.c_uint64, ctypes.POINTER(i32)]),
        "fri_commit_degrees": (i32, [vp, ctypes.POINTER(ctypes.c_int32), sz, ctypes.POINTER(u32)]),
        "fri_debug_transport_log": (i32, [vp, ctypes.POINTER(TransportOp), sz, ctypes.POINTER(sz)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _u32(a) -> np.ndarray:
    if isinstance(a, np.ndarray) and a.dtype == np.uint32:
        # no widening copy: every library entry point checks canonicity itself
        # (FRI_EINVAL, raised by _check); the uint64 round trip below cost
        # about 1.5 ms per 2^21 coefficients
        return np.ascontiguousarray(a)
    arr = np.ascontiguousarray(np.asarray(a, dtype=np.uint64))
    if arr.size and int(arr.max()) >= P:
        raise FriError(FRI_EINVAL, "field element not canonical (>= p)")
    return np.ascontiguousarray(arr.astype(np.uint32))


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))


class Context:
    """Owns one fri_ctx (device buffers, stream, graphs) on one GPU, or, from
    ``Context.multi``, a team of ranks on several GPUs behind one context."""

    def __init__(self, device: int = 0, log_n_max: int = 20, _handle=None, _owner=True):
        self.lib = load_library()
        self.device = device
        self.log_n_max = log_n_max
        self.n_ranks = 1
        self._owner = _owner
        if _handle is not None:
            self.h = _handle
            return
        h = ctypes.c_void_p()
        rc = self.lib.fri_ctx_create(device, log_n_max, ctypes.byref(h))
        if rc != FRI_OK:
            raise FriError(rc, "fri_ctx_create failed (no gfx950 device?)")
        self.h = h

    @classmethod
    def multi(cls, devices: Sequence[int], log_n_max: int, transport: str = "auto") -> "Context":
        """fri_ctx_create_multi: ONE context over len(devices) GPUs (ranks;
        a device may repeat), driven from this thread.  commit / commit_device
        of a codeword >= 2^20 run coset-sharded over the ranks in one call;
        every read-back serves the whole commit.  transport: "auto" (the
        peer transport), "peer" or "rccl" (opt-in, distinct devices only)."""
        lib = load_library()
        kinds = {"auto": 0, "rccl": 1, "peer": 4}
        if transport not in kinds:
            raise FriError(FRI_EINVAL, f"transport must be one of {sorted(kinds)}")
        devs = (ctypes.c_int * len(devices))(*[int(x) for x in devices])
        h = ctypes.c_void_p()
        rc = lib.fri_ctx_create_multi(devs, len(devices), log_n_max, kinds[transport], ctypes.byref(h))
        if rc != FRI_OK:
            raise FriError(rc, f"fri_ctx_create_multi({list(devices)}, {log_n_max}, {transport}) failed")
        c = cls(int(devices[0]), log_n_max, _handle=h)
        c.n_ranks = len(devices)
        c.devices = [int(x) for x in devices]
        return c

    @classmethod
    def default(cls, log_n_max: int) -> "Context":
        """fri_ctx_create_default: the devices named by FRI_DEVICES (e.g.
        "0,0,0,0"), else every visible GPU (largest power-of-two count); one
        device is an ordinary context, several a team (peer transport, or
        FRI_TRANSPORT=rccl).  What the reference-shaped functions below use
        when no ctx is passed."""
        lib = load_library()
        h = ctypes.c_void_p()
        n = ctypes.c_uint32()
        rc = lib.fri_ctx_create_default(log_n_max, ctypes.byref(h), ctypes.byref(n))
        if rc != FRI_OK:
            raise FriError(rc, f"fri_ctx_create_default({log_n_max}) failed (FRI_DEVICES="
                               f"{os.environ.get('FRI_DEVICES', '')!r}; no gfx950 device?)")
        c = cls(0, log_n_max, _handle=h)
        c.n_ranks = n.value
        return c

    def input_buffer(self, d: int) -> int:
        """Device pointer of the context's input buffer (fri_ctx_input_buffer):
        the caller's; no commit writes it, commits from it read it in place."""
        p = ctypes.c_void_p()
        self._check(self.lib.fri_ctx_input_buffer(self.h, d, ctypes.byref(p)))
        return p.value

    def input_upload(self, coeffs) -> int:
        """Fill the input buffer with host coefficients (fri_ctx_input_upload;
        waits for the pending commits reading it) and return its pointer."""
        c = _u32(coeffs)
        self._check(self.lib.fri_ctx_input_upload(self.h, _ptr(c), c.size))
        return self.input_buffer(c.size)

    def force_copy(self, enable: bool = True):
        """Test hook (fri_debug_team_force_copy): a team's collectives copy with
        hipMemcpyPeerAsync per source instead of the pull kernel."""
        self._check(self.lib.fri_debug_team_force_copy(self.h, 1 if enable else 0))

    def team_rank(self, rank: int) -> "Context":
        """A non-owning view of rank ``rank``'s context (fri_debug_team_rank),
        for its transport log and device bytes."""
        h = ctypes.c_void_p()
        self._check(self.lib.fri_debug_team_rank(self.h, rank, ctypes.byref(h)))
        return Context(self.device, self.log_n_max, _handle=h, _owner=False)

    def inject_team_failure(self, rank: int, op_index: int):
        """Test hook (fri_debug_team_inject_failure): rank `rank` fails its
        op_index-th collective in the next team call."""
        self._check(self.lib.fri_debug_team_inject_failure(self.h, rank, op_index))

    def close(self):
        if self.h and self._owner:
            self.lib.fri_ctx_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int):
        if rc != FRI_OK:
            raise FriError(rc, self.lib.fri_last_error(self.h).decode())

    # ---- kernel-level ops ------------------------------------------------
    def batch_inverse(self, xs) -> np.ndarray:
        a = _u32(xs)
        out = np.empty_like(a)
        self._check(self.lib.fri_batch_inverse(self.h, _ptr(a), _ptr(out), a.size))
        return out

    def lde(self, coeffs, log_n: int, offset: int = GENERATOR) -> np.ndarray:
        c = _u32(coeffs)
        out = np.empty(1 << log_n, dtype=np.uint32)
        self._check(self.lib.fri_lde(self.h, _ptr(c), c.size, log_n, offset, _ptr(out)))
        return out

    def interpolate(self, ys, offset: int = GENERATOR) -> np.ndarray:
        y = _u32(ys)
        log_n = int(y.size).bit_length() - 1
        if y.size != 1 << log_n:
            raise FriError(FRI_EINVAL, "coset interpolation needs a power-of-two point count")
        out = np.empty(y.size, dtype=np.uint32)
        ln = ctypes.c_size_t()
        self._check(self.lib.fri_interpolate(self.h, _ptr(y), log_n, offset, _ptr(out), ctypes.byref(ln)))
        return out[: ln.value]

    def interpolate_points(self, xs, ys) -> np.ndarray:
        """Polynomial::interpolate(xs, ys) on arbitrary points
        (interpolation.rs:121-152; fri_interpolate_points), trimmed."""
        x, y = _u32(xs), _u32(ys)
        if x.size != y.size:
            raise FriError(FRI_EINVAL, "Mismatched x and y lengths")   # interpolation.rs:127-133 panics
        out = np.empty(max(1, x.size), dtype=np.uint32)
        ln = ctypes.c_size_t()
        self._check(self.lib.fri_interpolate_points(self.h, _ptr(x), _ptr(y), x.size, _ptr(out), ctypes.byref(ln)))
        return out[: ln.value]

    def evaluate(self, coeffs, xs) -> np.ndarray:
        c, x = _u32(coeffs), _u32(xs)
        out = np.empty(x.size, dtype=np.uint32)
        self._check(self.lib.fri_evaluate(self.h, _ptr(c), c.size, _ptr(x), x.size, _ptr(out)))
        return out

    def fold(self, layer, layer_offset: int, beta: int) -> np.ndarray:
        v = _u32(layer)
        log_m = int(v.size).bit_length() - 1
        out = np.empty(v.size // 2, dtype=np.uint32)
        self._check(self.lib.fri_fold(self.h, _ptr(v), log_m, layer_offset, beta, _ptr(out)))
        return out

    def merkle_root(self, values) -> bytes:
        v = _u32(values)
        root = ctypes.create_string_buffer(32)
        self._check(self.lib.fri_merkle_root(self.h, _ptr(v), v.size, root))
        return root.raw

    # ---- commit ----------------------------------------------------------
    def commit(self, coeffs, log_n: int, offset: int = GENERATOR, channel_state: Optional[bytes] = None,
               forced_betas: Optional[Sequence[int]] = None, graph: bool = True) -> CommitResult:
        c = _u32(coeffs)
        ch = ChannelState()
        if channel_state:
            ctypes.memmove(ch.digest, channel_state, 32)
            ch.has_state = 1
        flags = 0 if graph else FLAG_NO_GRAPH
        fb = None
        if forced_betas is not None:
            fbarr = np.zeros(MAX_ROUNDS, dtype=np.uint32)
            fbarr[: len(forced_betas)] = forced_betas
            fb = fbarr
            flags |= FLAG_FORCE_BETAS
        res = CommitResult()
        self._check(self.lib.fri_commit(self.h, _ptr(c), c.size, log_n, offset, ctypes.byref(ch), flags,
                                        _ptr(fb) if fb is not None else None, ctypes.byref(res)))
        return res

    def commit_device_async(self, d_coeffs, d: int, log_n: int, offset: int = GENERATOR,
                            channel_state: Optional[bytes] = None) -> int:
        """Enqueue a commit of device-resident coefficients (``d_coeffs``: a
        device pointer, e.g. from fri_ctx_input_buffer) and return its ticket
        at once (fri_commit_device_async; at most MAX_INFLIGHT pending)."""
        ch = ChannelState()
        if channel_state:
            ctypes.memmove(ch.digest, channel_state, 32)
            ch.has_state = 1
        t = ctypes.c_uint64()
        self._check(self.lib.fri_commit_device_async(self.h, d_coeffs, d, log_n, offset, ctypes.byref(ch), 0, None,
                                                     ctypes.byref(t)))
        return t.value

    def commit_async(self, coeffs, log_n: int, offset: int = GENERATOR,
                     channel_state: Optional[bytes] = None) -> int:
        """Enqueue a commit of host coefficients and return its ticket
        (fri_commit_async: the coefficients are copied before it returns)."""
        c = _u32(coeffs)
        ch = ChannelState()
        if channel_state:
            ctypes.memmove(ch.digest, channel_state, 32)
            ch.has_state = 1
        t = ctypes.c_uint64()
        self._check(self.lib.fri_commit_async(self.h, _ptr(c), c.size, log_n, offset, ctypes.byref(ch), 0, None,
                                              ctypes.byref(t)))
        return t.value

    def set_lanes(self, max_lanes: int):
        """Commit lanes of the pipelined commits (fri_ctx_set_lanes): each
        pending commit runs on the lane with the fewest pending commits, each
        lane a stream with its own plan, so consecutive commits overlap."""
        self._check(self.lib.fri_ctx_set_lanes(self.h, max_lanes))

    def ticket_lane(self, ticket: int) -> int:
        """Lane a pending pipelined commit was dealt to (fri_debug_ticket_lane)."""
        lane = ctypes.c_int()
        self._check(self.lib.fri_debug_ticket_lane(self.h, ticket, ctypes.byref(lane)))
        return lane.value

    def commit_wait(self, ticket: int, out: Optional[CommitResult] = None) -> CommitResult:
        """Wait for an enqueued commit and return its result (fri_commit_wait)."""
        res = out if out is not None else CommitResult()
        self._check(self.lib.fri_commit_wait(self.h, ticket, ctypes.byref(res)))
        return res

    def commit_info(self):
        """(generation, log_n, n_layers) of the resident commit (fri_commit_info)."""
        g, ln, nl = ctypes.c_uint64(), ctypes.c_uint32(), ctypes.c_uint32()
        self._check(self.lib.fri_commit_info(self.h, ctypes.byref(g), ctypes.byref(ln), ctypes.byref(nl)))
        return g.value, ln.value, nl.value

    def _resident(self, log_n: int, generation: Optional[int] = None) -> None:
        """Read-backs serve only the commit they were asked for: the resident
        codeword must be 2^log_n and, for a FRIProof, still the commit of
        ``generation`` (a later commit on this context replaced its layers)."""
        g, ln, nl = self.commit_info()
        if generation is not None and g != generation:
            raise FriError(FRI_ESTATE, "FRIProof layers were replaced by a later commit on the same context")
        if nl and ln != log_n:
            raise FriError(FRI_ESTATE, f"resident commit is 2^{ln}, not 2^{log_n}")

    def layer(self, k: int, log_n: int, generation: Optional[int] = None) -> np.ndarray:
        self._resident(log_n, generation)
        out = np.empty(1 << (log_n - k), dtype=np.uint32)
        self._check(self.lib.fri_layer_copy(self.h, k, _ptr(out), out.size))
        return out

    def tree_level(self, k: int, level: int, log_n: int) -> List[bytes]:
        self._resident(log_n)
        cnt = 1 << (log_n - k - level)
        buf = ctypes.create_string_buffer(32 * cnt)
        self._check(self.lib.fri_tree_level_copy(self.h, k, level, buf, 32 * cnt))
        raw = buf.raw
        return [raw[32 * i: 32 * i + 32] for i in range(cnt)]

    def auth_path(self, k: int, index: int, log_n: int):
        self._resident(log_n)
        depth = log_n - k
        buf = ctypes.create_string_buffer(32 * max(depth, 1))
        val = ctypes.c_uint32()
        dep = ctypes.c_uint32()
        self._check(self.lib.fri_auth_path(self.h, k, index, ctypes.byref(val), buf, ctypes.byref(dep)))
        return val.value, [buf.raw[32 * i: 32 * i + 32] for i in range(dep.value)]

    def trace_commit(self, trace, log_blowup: int, offset: int = GENERATOR, readback: bool = True):
        """fri_trace_commit: (LDE Merkle root bytes, trimmed trace-polynomial
        coefficients, LDE values) for 2^log_t trace values (coefficients and
        LDE are None with readback=False: they stay on the device)."""
        tr = _u32(trace)
        log_t = tr.size.bit_length() - 1
        if tr.size != 1 << log_t:
            raise FriError(FRI_EINVAL, "trace length must be a power of two")
        root = ctypes.create_string_buffer(32)
        if not readback:
            self._check(self.lib.fri_trace_commit(self.h, _ptr(tr), log_t, log_blowup, offset, root, None, None,
                                                  None))
            return root.raw, None, None
        coeffs = np.empty(tr.size, dtype=np.uint32)
        lde = np.empty(tr.size << log_blowup, dtype=np.uint32)
        ln = ctypes.c_size_t()
        self._check(self.lib.fri_trace_commit(self.h, _ptr(tr), log_t, log_blowup, offset, root, _ptr(coeffs),
                                              ctypes.byref(ln), _ptr(lde)))
        return root.raw, coeffs[: ln.value], lde

    def fibsq_composition_commit(self, log_t: int, log_blowup: int, a_last: int, alphas: Sequence[int],
                                 offset: int = GENERATOR, channel_state: Optional[bytes] = None,
                                 graph: bool = True) -> CommitResult:
        """fri_fibsq_composition_commit: composition polynomial of the resident
        trace LDE, then the FRI commit of it (channel continued from
        ``channel_state``)."""
        al = _u32(alphas)
        if al.size != 3:
            raise FriError(FRI_EINVAL, "three alphas")
        ch = ChannelState()
        if channel_state:
            ctypes.memmove(ch.digest, channel_state, 32)
            ch.has_state = 1
        res = CommitResult()
        self._check(self.lib.fri_fibsq_composition_commit(self.h, log_t, log_blowup, offset, a_last, _ptr(al),
                                                          ctypes.byref(ch), 0 if graph else FLAG_NO_GRAPH,
                                                          ctypes.byref(res)))
        return res

    def trace_decommit(self, index: int, stride: int, count: int, depth: int):
        """fri_trace_decommit: [(LDE[index + j*stride], path bytes)] for j < count."""
        vals = np.empty(count, dtype=np.uint32)
        buf = ctypes.create_string_buffer(32 * depth * count)
        self._check(self.lib.fri_trace_decommit(self.h, index, stride, count, _ptr(vals), buf, len(buf)))
        pl = 32 * depth
        return [(int(vals[j]), buf.raw[j * pl:(j + 1) * pl]) for j in range(count)]

    def decommit_query(self, index: int, n_layers: int, log_n: int, generation: Optional[int] = None,
                       sharded: bool = False):
        """fri_decommit_query: per committed layer k, (value[idx], value[sib],
        path(idx), path(sib)) with idx = index % m_k, sib = (idx + m_k/2) % m_k.
        sharded: after commit_sharded, fri_decommit_query_sharded (collective:
        every rank calls it with the same index)."""
        self._resident(log_n, generation)
        if n_layers != self.commit_info()[2]:
            raise FriError(FRI_ESTATE, "layer count differs from the resident commit")
        vals = np.empty(2 * n_layers, dtype=np.uint32)
        total = sum(64 * (log_n - k) for k in range(n_layers))
        buf = ctypes.create_string_buffer(max(total, 1))
        ln = ctypes.c_size_t()
        fn = self.lib.fri_decommit_query_sharded if sharded else self.lib.fri_decommit_query
        self._check(fn(self.h, index, _ptr(vals), vals.size, buf, total, ctypes.byref(ln)))
        out, off = [], 0
        for k in range(n_layers):
            pl = 32 * (log_n - k)
            out.append((int(vals[2 * k]), int(vals[2 * k + 1]), buf.raw[off:off + pl], buf.raw[off + pl:off + 2 * pl]))
            off += 2 * pl
        return out

    # ---- multi-GPU ---------------------------------------------------------
    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(128)
        rc = load_library().fri_dist_unique_id(buf)
        if rc != FRI_OK:
            raise FriError(rc, "ncclGetUniqueId failed")
        return buf.raw

    def attach_rccl(self, rank: int, world: int, uid: bytes):
        self._check(self.lib.fri_dist_attach_rccl(self.h, rank, world, uid))

    def attach_torch(self, rank: int, world: int):
        """Host-staged collectives over the default torch.distributed group
        (gloo on CPU tensors): used to run the sharded path with several
        ranks on one GPU (tests)."""
        import torch
        import torch.distributed as dist

        def as_np(ptr, nbytes):
            return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint8)), shape=(nbytes,))

        def allgather(user, send, recv, b):
            try:
                src = torch.from_numpy(as_np(send, b).copy())
                outs = [torch.empty(b, dtype=torch.uint8) for _ in range(world)]
                dist.all_gather(outs, src)
                dst = as_np(recv, b * world)
                for r in range(world):
                    dst[r * b:(r + 1) * b] = outs[r].numpy()
                return 0
            except Exception:  # noqa: BLE001
                return 1

        def alltoall(user, send, recv, b):
            try:
                src = torch.from_numpy(as_np(send, b * world).copy())
                out = torch.empty(b * world, dtype=torch.uint8)
                dist.all_to_all_single(out, src)
                as_np(recv, b * world)[:] = out.numpy()
                return 0
            except Exception:  # noqa: BLE001
                return 1

        def sendrecv(user, send, recv, b, peer):
            try:
                src = torch.from_numpy(as_np(send, b).copy())
                out = torch.empty(b, dtype=torch.uint8)
                ops = [dist.P2POp(dist.isend, src, peer), dist.P2POp(dist.irecv, out, peer)]
                for r in dist.batch_isend_irecv(ops):
                    r.wait()
                as_np(recv, b)[:] = out.numpy()
                return 0
            except Exception:  # noqa: BLE001
                return 1

        t = Collectives._fields_
        self._cb = Collectives(None, t[1][1](allgather), t[2][1](alltoall), t[3][1](sendrecv))
        self._check(self.lib.fri_dist_attach_host(self.h, rank, world, ctypes.byref(self._cb)))

    def attach_loopback(self, rank: int, world: int):
        """Timing rehearsal (fri_debug_attach_loopback): collectives return
        this rank's own bytes; the transcript is not the real one."""
        self._check(self.lib.fri_debug_attach_loopback(self.h, rank, world))

    def loopback_degrees(self, degrees: Optional[Sequence[int]]):
        """The rehearsal's degree schedule (fri_debug_loopback_degrees): the
        per-layer degrees of a 1-GPU commit of the same polynomial
        (commit_degrees), so the rehearsal runs every round of the real
        commit although the coefficient fold is sharded. None clears it."""
        if not degrees:
            self._check(self.lib.fri_debug_loopback_degrees(self.h, None, 0))
            return
        a = (ctypes.c_int32 * len(degrees))(*[int(x) for x in degrees])
        self._check(self.lib.fri_debug_loopback_degrees(self.h, a, len(degrees)))

    def commit_degrees(self) -> List[int]:
        """deg(poly_k) of every layer of the resident commit (fri_commit_degrees)."""
        n = ctypes.c_uint32()
        buf = (ctypes.c_int32 * (MAX_ROUNDS + 1))()
        self._check(self.lib.fri_commit_degrees(self.h, buf, MAX_ROUNDS + 1, ctypes.byref(n)))
        return [int(buf[i]) for i in range(n.value)]

    def transport_log(self) -> List[tuple]:
        """(chan, op, peer, bytes) of every collective of the last sharded call
        (fri_debug_transport_log); op is "allgather", "alltoall" or "sendrecv"."""
        cnt = ctypes.c_size_t()
        self._check(self.lib.fri_debug_transport_log(self.h, None, 0, ctypes.byref(cnt)))
        buf = (TransportOp * max(1, cnt.value))()
        self._check(self.lib.fri_debug_transport_log(self.h, buf, cnt.value, ctypes.byref(cnt)))
        return [(e.chan, TRANSPORT_OPS[e.op], e.peer, e.bytes) for e in buf[:cnt.value]]

    def detach(self):
        self._check(self.lib.fri_dist_detach(self.h))

    def dist_info(self):
        """(rank, world, transport) as the attached transport reports them
        (transport: "none", "rccl", "host", "loopback" or "peer"; fri_dist_info)."""
        r, w, t = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        self._check(self.lib.fri_dist_info(self.h, ctypes.byref(r), ctypes.byref(w), ctypes.byref(t)))
        return r.value, w.value, TRANSPORTS[t.value]

    def dist_selftest(self, words_per_peer: int = 4096):
        self._check(self.lib.fri_dist_selftest(self.h, words_per_peer))

    def commit_sharded(self, coeffs, log_n: int, offset: int = GENERATOR, channel_state: Optional[bytes] = None,
                       forced_betas: Optional[Sequence[int]] = None) -> CommitResult:
        c = _u32(coeffs)
        ch = ChannelState()
        if channel_state:
            ctypes.memmove(ch.digest, channel_state, 32)
            ch.has_state = 1
        flags, fb = 0, None
        if forced_betas is not None:
            fb = np.zeros(MAX_ROUNDS, dtype=np.uint32)
            fb[: len(forced_betas)] = forced_betas
            flags |= FLAG_FORCE_BETAS
        res = CommitResult()
        self._check(self.lib.fri_commit_sharded(self.h, _ptr(c), c.size, log_n, offset, ctypes.byref(ch), flags,
                                                _ptr(fb) if fb is not None else None, ctypes.byref(res)))
        return res

    def set_profiling(self, on: bool):
        self._check(self.lib.fri_set_profiling(self.h, 1 if on else 0))

    def profile(self, cls: str):
        ms, n, b = ctypes.c_double(), ctypes.c_uint64(), ctypes.c_uint64()
        self._check(self.lib.fri_get_profile(self.h, cls.encode(), ctypes.byref(ms), ctypes.byref(n),
                                             ctypes.byref(b)))
        return ms.value, n.value, b.value

    def reset_profile(self):
        self._check(self.lib.fri_reset_profile(self.h))

    def set_device_cap(self, cap_bytes: int):
        """Test hook (fri_debug_set_device_cap): device allocations of this
        context beyond cap_bytes fail as out-of-memory; 0 removes the cap."""
        self._check(self.lib.fri_debug_set_device_cap(self.h, cap_bytes))

    def device_bytes(self):
        """(current, peak) HBM bytes held by this context (fri_ctx_device_bytes)."""
        cur, peak = ctypes.c_uint64(), ctypes.c_uint64()
        self._check(self.lib.fri_ctx_device_bytes(self.h, ctypes.byref(cur), ctypes.byref(peak)))
        return cur.value, peak.value


_HIP = None


def hip_runtime() -> ctypes.CDLL:
    """The HIP runtime libfri_amd.so is linked against (loaded with it): for
    a caller's own device buffers without a second runtime in the process
    (PyTorch bundles its own libamdhip64)."""
    global _HIP
    if _HIP is not None:
        return _HIP
    load_library()
    path = "libamdhip64.so.7"
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if "libamdhip64.so" in line and "/torch/" not in line:
                    path = line.split()[-1]
                    break
    except OSError:
        pass
    hip = ctypes.CDLL(path)
    vp = ctypes.c_void_p
    hip.hipMalloc.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t]
    hip.hipFree.argtypes = [vp]
    hip.hipStreamCreate.argtypes = [ctypes.POINTER(vp)]
    hip.hipStreamDestroy.argtypes = [vp]
    hip.hipStreamSynchronize.argtypes = [vp]
    hip.hipMemcpyAsync.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int, vp]
    _HIP = hip
    return hip


class DeviceBuffer:
    """A device copy of a uint32 array for fri_commit_device /
    fri_commit_device_async (hipMalloc, then an upload on a stream of its own,
    so the null stream never takes one of the process's hardware queues);
    freed with the object.  ``data_ptr()`` is the device pointer."""

    def __init__(self, arr):
        a = np.ascontiguousarray(arr, dtype=np.uint32)
        hip = hip_runtime()
        self._hip = hip
        p = ctypes.c_void_p()
        if hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(max(4, a.nbytes))) != 0:
            raise FriError(FRI_ENOMEM, "hipMalloc of a device buffer failed")
        self.ptr = p.value
        st = ctypes.c_void_p()
        if (hip.hipStreamCreate(ctypes.byref(st)) != 0 or
                hip.hipMemcpyAsync(p, a.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(a.nbytes), 1, st) != 0 or
                hip.hipStreamSynchronize(st) != 0):
            raise FriError(FRI_EHIP, "upload of a device buffer failed")
        hip.hipStreamDestroy(st)

    def data_ptr(self) -> int:
        return self.ptr

    def __del__(self):
        if getattr(self, "ptr", None):
            self._hip.hipFree(self.ptr)
            self.ptr = None


def plan_layout(d: int, log_n: int, world: int = 1, rank: int = 0) -> dict:
    """The commit plan's layout (fri_debug_plan_layout; host only, no GPU):
    rounds bound, last sharded layer, per-layer slot sizes, x^-1 slices and
    the block the rank holds."""
    cap = 4 + 5 * (MAX_ROUNDS + 1)
    out = (ctypes.c_uint64 * cap)()
    rc = load_library().fri_debug_plan_layout(d, log_n, world, rank, out, cap)
    if rc != FRI_OK:
        raise FriError(rc, "fri_debug_plan_layout")
    rmax = int(out[0])
    layers = [dict(zip(("layer_words", "tree_words", "xinv_count", "xinv_start", "block"),
                       (int(x) for x in out[4 + 5 * k: 9 + 5 * k]))) for k in range(rmax + 1)]
    k_sw = int(out[1])
    return {"rmax": rmax, "k_sw": k_sw - (1 << 64) if k_sw >= 1 << 63 else k_sw, "bytes": int(out[2]),
            "coef_chunk_log2": int(out[3]), "layers": layers}


# ----------------------------------------------------------------------------
# Reference-shaped host objects
# ----------------------------------------------------------------------------
@dataclass
class Channel:
    """src/channel/channel.rs — host-side transcript (authoritative state).

    fri_commit() hands the state to the device, which replays the exact same
    send/receive sequence, and then appends the same proof messages here."""
    state: str = ""
    proof: List[bytes] = field(default_factory=list)
    compressed_proof: List[bytes] = field(default_factory=list)

    def send(self, message: bytes) -> None:                               # channel.rs:35-44
        self.state = hashlib.sha256((self.state + bytes(message).hex()).encode()).hexdigest()
        self.proof.append(bytes(message))
        self.compressed_proof.append(bytes(message))

    def receive_random_int(self, lo: int, hi: int, show_in_proof: bool) -> int:   # channel.rs:58-84
        if not self.state:
            raise FriError(FRI_ESTATE, "Channel state is not valid hex")   # channel.rs:65
        num = (int(self.state, 16) + lo) % ((hi - lo) + 1)
        self.state = hashlib.sha256(self.state.encode()).hexdigest()
        num &= (1 << 64) - 1
        if show_in_proof:
            self.proof.append(num.to_bytes(8, "big"))
        return num

    def receive_random_field_element(self) -> int:                        # channel.rs:47-55
        num = self.receive_random_int(0, P - 1, False)
        self.proof.append(num.to_bytes(8, "big"))
        return num % P

    def proof_size(self) -> int:                                          # channel.rs:88-90
        return sum(len(b) for b in self.proof)

    def compressed_proof_size(self) -> int:                               # channel.rs:93-95
        return sum(len(b) for b in self.compressed_proof)


class MerkleTree:
    """src/merkle/mod.rs:5-27 — SHA-256 tree over u64-BE leaves (GPU-built).
    A standalone tree keeps its root; the trees of an FRIProof
    (``FRIProof.fri_merkles``) are the device-resident ones of that commit
    and also serve authentication paths."""

    def __init__(self, values: Sequence[int], ctx: Optional[Context] = None):
        self._ctx = ctx or _default_ctx(max(1, (len(values) - 1).bit_length()))
        self._root = self._ctx.merkle_root(values)
        self._generation = None
        self._layer = None
        self._log_n = None
        self._sharded = False

    @classmethod
    def _on_device(cls, ctx: Context, generation: int, layer: int, log_n: int, root: bytes,
                   sharded: bool = False) -> "MerkleTree":
        t = cls.__new__(cls)
        t._ctx, t._root, t._generation, t._layer, t._log_n = ctx, root, generation, layer, log_n
        t._sharded = sharded
        return t

    def root(self) -> str:
        return self._root.hex()

    def get_authentication_path(self, idx: int) -> bytes:
        """rs_merkle single-leaf proof of leaf idx (sibling digests leaf ->
        root) from the device-resident tree (fri_auth_path)."""
        if self._generation is None:
            raise FriError(FRI_ESTATE, "a standalone tree keeps only its root")
        self._ctx._resident(self._log_n, self._generation)
        _, path = self._ctx.auth_path(self._layer, idx, self._log_n)
        return b"".join(path)


@dataclass
class FRIProof:
    """src/fri/fri_commit.rs:9-13 — layers/merkles read back lazily from the device."""
    ctx: Context
    log_n: int
    roots: List[bytes]
    betas: List[int]
    final_value: int
    final_degree: int
    generation: int = 0      # fri_commit_info generation of the commit that made it
    sharded: bool = False    # made by fri_commit_sharded: decommitments are collective

    @property
    def n_layers(self) -> int:
        return len(self.roots)

    def layer(self, k: int) -> np.ndarray:
        return self.ctx.layer(k, self.log_n, self.generation)

    @property
    def fri_layers(self) -> List[np.ndarray]:
        return [self.layer(k) for k in range(self.n_layers)]

    def merkle_root(self, k: int) -> str:
        return self.roots[k].hex()

    @property
    def fri_merkles(self) -> List[MerkleTree]:
        """FRIProof.fri_merkles (fri_commit.rs:9-13): the commit's trees, device-backed."""
        return [MerkleTree._on_device(self.ctx, self.generation, k, self.log_n, r, self.sharded)
                for k, r in enumerate(self.roots)]

    @property
    def final_poly(self) -> List[int]:
        return [] if self.final_degree == -1 else [self.final_value]


def decommit_fri_layers(index: int, proof: "FRIProof", channel: Channel) -> None:
    """src/fri/fri_commit.rs:137-163 over the device-resident layers/trees:
    per layer send value, path, sibling value, sibling path (a 1-element
    layer first sends its value, as the reference does)."""
    _send_openings(proof.ctx.decommit_query(index, proof.n_layers, proof.log_n, proof.generation, proof.sharded),
                   channel)


def _send_openings(openings, channel: Channel) -> None:
    for val, sval, path, spath in openings:
        # the gather reads layers of 2^(log_n-k) >= 2 elements; a 1-element
        # layer (blowup 1) has idx = sib = 0 and empty paths
        if not path and not spath:
            channel.send(val.to_bytes(8, "big"))
        channel.send(val.to_bytes(8, "big"))
        channel.send(path)
        channel.send(sval.to_bytes(8, "big"))
        channel.send(spath)


def decommit_fri(num_queries: int, max_index: int, proof, merkles_or_channel, channel: Optional[Channel] = None) -> None:
    """src/fri/fri_commit.rs:168-179: each index drawn with
    receive_random_int(0, max_index, true) from the transcript so far.
    Two forms: decommit_fri(q, max, proof, channel), or the reference's own
    decommit_fri(q, max, fri_layers, fri_merkles, channel) with the proof's
    ``fri_layers`` and device-backed ``fri_merkles`` (the commit is found
    through the trees; their generation must still be resident, and the
    openings must equal ``fri_layers``)."""
    if channel is None:
        for _ in range(num_queries):
            idx = merkles_or_channel.receive_random_int(0, max_index, True)
            decommit_fri_layers(idx, proof, merkles_or_channel)
        return
    layers, merkles = proof, merkles_or_channel
    if not merkles or len(layers) != len(merkles):
        raise FriError(FRI_EINVAL, "one Merkle tree per FRI layer")
    t0 = merkles[0]
    if t0._generation is None or any(t._ctx is not t0._ctx or t._generation != t0._generation or t._layer != k
                                     for k, t in enumerate(merkles)):
        raise FriError(FRI_EINVAL, "fri_merkles are not the device-backed trees of one commit")
    ctx, log_n = t0._ctx, t0._log_n
    for _ in range(num_queries):
        idx = channel.receive_random_int(0, max_index, True)
        openings = ctx.decommit_query(idx, len(merkles), log_n, t0._generation, t0._sharded)
        for k, (v, sv, _, _) in enumerate(openings):
            m = 1 << (log_n - k)
            i = idx % m
            if len(layers[k]) != m or int(layers[k][i]) != v or int(layers[k][(i + m // 2) % m]) != sv:
                raise FriError(FRI_ESTATE, f"fri_layers do not belong to the commit of these fri_merkles (layer {k})")
        _send_openings(openings, channel)


def _merkle_path_ok(value: int, index: int, path: bytes, depth: int, root: bytes) -> bool:
    """rs_merkle single-leaf proof of a power-of-two tree: siblings leaf -> root."""
    if len(path) != 32 * depth:
        return False
    h = hashlib.sha256(value.to_bytes(8, "big")).digest()              # merkle/mod.rs:14-15
    for lvl in range(depth):
        sib = path[32 * lvl:32 * lvl + 32]
        h = hashlib.sha256(sib + h if (index >> lvl) & 1 else h + sib).digest()
    return h == root


def verify_fri(messages: Sequence[bytes], log_n: int, n_layers: int, num_queries: int, max_index: int,
               offset: int = GENERATOR, channel_state: str = "") -> bool:
    """Check a FRI transcript: the proof messages that fri_commit followed by
    decommit_fri append to Channel.proof (fri_commit.rs:72-179).

    The reference's verify_fri (src/fri/fri_verify.rs:12-177) is a sketch.
    It re-reads proof.last() and leaves the fold check as a placeholder, so
    this is the check it outlines, made complete:
      * replay a fresh channel from ``channel_state``: every root is sent;
        every beta and query index must be the one the replay draws; the
        final value is sent;
      * every authentication path must lead to its layer's root;
      * every layer k >= 1 value must equal the fold of its two parents:
        (a + b)/2 + beta (a - b) / (2 x);
      * the last layer must hold the final constant.
    ``n_layers`` = number of committed layers (the reference's
    expected_num_layers). Returns False on any mismatch or malformed transcript.
    """
    return _verify_transcript(messages, log_n, n_layers, num_queries, max_index, offset, channel_state)


class _Reject(Exception):
    pass


def _verify_transcript(messages, log_n, n_layers, num_queries, max_index, offset, channel_state,
                       pre_commit=None, on_query=None) -> bool:
    """verify_fri's replay with two hooks for a STARK around the FRI:
    ``pre_commit(take, ch)`` consumes the messages before the first FRI root;
    ``on_query(take, ch, idx)`` those between a query index and its layer
    openings, and returns the value layer 0 must hold at idx (or None)."""
    msgs = list(messages)
    pos = 0

    def take():
        nonlocal pos
        if pos >= len(msgs):
            raise ValueError("transcript ended early")
        pos += 1
        return msgs[pos - 1]

    try:
        ch = Channel(state=channel_state)
        if pre_commit is not None:
            pre_commit(take, ch)
        roots, betas = [], []
        for k in range(n_layers):
            r = take()
            if len(r) != 64:
                return False
            roots.append(bytes.fromhex(r.decode()))
            ch.send(r)
            if k < n_layers - 1:
                beta = ch.receive_random_field_element()
                if take() != beta.to_bytes(8, "big"):
                    return False
                betas.append(beta)
        fin = take()
        if len(fin) != 8:
            return False
        final = int.from_bytes(fin, "big")
        ch.send(fin)
        inv2 = pow(2, P - 2, P)
        for _ in range(num_queries):
            idx = ch.receive_random_int(0, max_index, True)
            if take() != idx.to_bytes(8, "big"):
                return False
            want0 = on_query(take, ch, idx) if on_query is not None else None
            prev = None                                  # (value at i, value at i + m/2, i, m) of layer k-1
            for k in range(n_layers):
                m = 1 << (log_n - k)
                depth = log_n - k
                extra = None
                if m == 1:
                    extra = take()                       # fri_commit.rs:147-149 sends layer[0] first
                    ch.send(extra)
                i = idx % m
                sib = (i + m // 2) % m
                vb, path, sb, spath = take(), take(), take(), take()
                if extra is not None and extra != vb:
                    return False
                for msg in (vb, path, sb, spath):
                    ch.send(msg)
                v, sv = int.from_bytes(vb, "big"), int.from_bytes(sb, "big")
                if v >= P or sv >= P:
                    return False
                if not (_merkle_path_ok(v, i, path, depth, roots[k]) and _merkle_path_ok(sv, sib, spath, depth, roots[k])):
                    return False
                if k == 0 and want0 is not None and v != want0:
                    return False
                if prev is not None:
                    pa, pb, pj, pm = prev                    # pa = L[pj], pb = L[pj + pm/2]
                    x = pow(offset, 1 << (k - 1), P) * pow(pow(GENERATOR, (P - 1) // pm, P), pj, P) % P
                    fold = ((pa + pb) + betas[k - 1] * (pa - pb) % P * pow(x, P - 2, P)) % P * inv2 % P
                    if fold != v:
                        return False
                j = i % (m // 2) if m > 1 else 0
                prev = (v, sv, j, m) if i < m // 2 or m == 1 else (sv, v, j, m)
                if k == n_layers - 1 and (v != final or sv != final):
                    return False
        return pos == len(msgs)
    except (ValueError, IndexError, UnicodeDecodeError, _Reject):
        return False


# ---- prover slice: STARK-101 FibonacciSq (BASELINE configs[3]) -------------
# src/prover, src/trace, src/composition are empty in the reference; the
# constraint system is STARK-101's (crate `stark-101`, Cargo.toml:2) on the
# full trace subgroup; see include/fri_amd.h (fri_fibsq_composition_commit).

def fibsq_trace(a1: int, T: int) -> np.ndarray:
    """a_0 = 1, a_1 = a1, a_{i+2} = a_{i+1}^2 + a_i^2 (mod p), T = 2^k rows
    (fri_fibsq_trace, host-side: the recurrence is one serial chain)."""
    log_t = T.bit_length() - 1
    if T != 1 << log_t:
        raise FriError(FRI_EINVAL, "trace length must be a power of two")
    out = np.empty(T, dtype=np.uint32)
    rc = load_library().fri_fibsq_trace(a1 % P, log_t, _ptr(out))
    if rc != FRI_OK:
        raise FriError(rc, "fri_fibsq_trace")
    return out


@dataclass
class StarkProof:
    trace_root: bytes
    alphas: List[int]
    a_last: int
    fri: FRIProof
    log_t: int
    log_blowup: int
    queries: List[int]


def prove_fibsq(a1: int, log_t: int, log_blowup: int, num_queries: int, channel: Channel,
                offset: int = GENERATOR, ctx: Optional[Context] = None) -> StarkProof:
    """STARK-101 prover on the GPU: trace -> LDE + Merkle (fri_trace_commit),
    send the trace root, draw alpha_0..2, composition polynomial + FRI commit
    (fri_fibsq_composition_commit), then per query (index drawn with
    receive_random_int(0, n - 2B - 1, true)) send f(x), f(gx), f(g^2 x) with
    their paths and the FRI layer openings (decommit_fri_layers,
    fri_commit.rs:137-163).  The transcript is ``channel.proof``."""
    L = log_t + log_blowup
    B, n = 1 << log_blowup, 1 << L
    ctx = ctx or _default_ctx(L)
    trace = fibsq_trace(a1, 1 << log_t)
    root, _, _ = ctx.trace_commit(trace, log_blowup, offset, readback=False)
    channel.send(root.hex().encode())
    alphas = [channel.receive_random_field_element() for _ in range(3)]
    res = ctx.fibsq_composition_commit(log_t, log_blowup, int(trace[-1]), alphas, offset,
                                       channel_state=bytes.fromhex(channel.state))
    fri = _mirror_commit(res, ctx, L, channel)
    queries = []
    for _ in range(num_queries):
        idx = channel.receive_random_int(0, n - 2 * B - 1, True)
        queries.append(idx)
        for v, path in ctx.trace_decommit(idx, B, 3, L):
            channel.send(v.to_bytes(8, "big"))
            channel.send(path)
        decommit_fri_layers(idx, fri, channel)
    return StarkProof(root, alphas, int(trace[-1]), fri, log_t, log_blowup, queries)


def fibsq_cp_at(f0: int, f1: int, f2: int, x: int, alphas: Sequence[int], a_last: int, log_t: int) -> int:
    """CP(x) from f(x), f(gx), f(g^2 x) (the composition the prover commits)."""
    T = 1 << log_t
    f0, f1, f2, x, a_last = int(f0), int(f1), int(f2), int(x), int(a_last)
    g = pow(GENERATOR, (P - 1) >> log_t, P)
    glast, gprev = pow(g, T - 1, P), pow(g, T - 2, P)
    p0 = (f0 - 1) * pow(x - 1, P - 2, P)
    p1 = (f0 - a_last) * pow(x - glast, P - 2, P)
    p2 = (f2 - f1 * f1 - f0 * f0) * (x - gprev) * (x - glast) * pow(pow(x, T, P) - 1, P - 2, P)
    return (alphas[0] * p0 + alphas[1] * p1 + alphas[2] * p2) % P


def verify_fibsq(messages: Sequence[bytes], a_last: int, log_t: int, log_blowup: int, num_queries: int,
                 n_layers: int, offset: int = GENERATOR, channel_state: str = "") -> bool:
    """Verifier of prove_fibsq's transcript: replays the channel (trace root,
    alphas, FRI roots/betas/final, query indices), checks every trace path
    against the trace root, that layer 0 at each query equals the composition
    polynomial computed from the opened f(x), f(gx), f(g^2 x), and then every
    FRI check of verify_fri."""
    L = log_t + log_blowup
    B, n = 1 << log_blowup, 1 << L
    a_last = int(a_last)
    state = {}

    def pre_commit(take, ch):
        r = take()
        if len(r) != 64:
            raise _Reject()
        state["root"] = bytes.fromhex(r.decode())
        ch.send(r)
        al = []
        for _ in range(3):
            a = ch.receive_random_field_element()
            if take() != a.to_bytes(8, "big"):
                raise _Reject()
            al.append(a)
        state["alphas"] = al

    def on_query(take, ch, idx):
        fs = []
        for j in range(3):
            vb, path = take(), take()
            ch.send(vb)
            ch.send(path)
            v = int.from_bytes(vb, "big")
            if len(vb) != 8 or v >= P or not _merkle_path_ok(v, idx + j * B, path, L, state["root"]):
                raise _Reject()
            fs.append(v)
        x = offset * pow(pow(GENERATOR, (P - 1) >> L, P), idx, P) % P
        return fibsq_cp_at(fs[0], fs[1], fs[2], x, state["alphas"], a_last, log_t)

    return _verify_transcript(messages, L, n_layers, num_queries, n - 2 * B - 1, offset, channel_state,
                              pre_commit, on_query)


_CTX_CACHE = {}


def _default_ctx(log_n: int) -> Context:
    """The context of the reference-shaped calls without ``ctx``: over the
    default devices (Context.default: FRI_DEVICES, else every visible GPU),
    at least 2^log_n (2^12 minimum), one per size bound, kept."""
    key = max(log_n, 12)
    for k, c in _CTX_CACHE.items():
        if k >= key:
            return c
    c = Context.default(key)
    _CTX_CACHE[key] = c
    return c


def fri_commit(coeffs: Sequence[int], log_n: int, channel: Channel, offset: int = GENERATOR,
               ctx: Optional[Context] = None) -> FRIProof:
    """src/fri/fri_commit.rs:72-122 on the coset domain offset*<w_{2^log_n}>.

    Updates ``channel`` exactly as the reference does: proof gets
    root_hex bytes per layer, 8-byte BE beta per round, 8-byte BE final value;
    state ends as the device computed it."""
    ctx = ctx or _default_ctx(log_n)
    st = bytes.fromhex(channel.state) if channel.state else None
    res = ctx.commit(coeffs, log_n, offset, channel_state=st)
    return _mirror_commit(res, ctx, log_n, channel)


def fri_commit_pipelined(polys: Sequence[Sequence[int]], log_n: int, channels: Sequence[Channel],
                         offset: int = GENERATOR, ctx=None, depth: int = DEFAULT_LANES) -> List[FRIProof]:
    """fri_commit (fri_commit.rs:72-122) of many polynomials in a row, each
    with its own channel, pipelined from this one host thread
    (fri_commit_async / fri_commit_wait, ``depth`` commits in flight per
    context, each on a commit lane of its own: one context overlaps them).
    ``ctx`` is one Context or a list of them: with several, the commits are
    dealt round-robin and run concurrently, one stream each.
    Proof i equals fri_commit of polys[i] into channels[i]; on each context
    only its last proof's layers stay resident."""
    if len(polys) != len(channels):
        raise FriError(FRI_EINVAL, "one channel per polynomial")
    if not 1 <= depth <= MAX_INFLIGHT:
        raise FriError(FRI_EINVAL, "depth must be 1..MAX_INFLIGHT")
    ctxs = list(ctx) if isinstance(ctx, (list, tuple)) else [ctx or _default_ctx(log_n)]
    if len({id(c) for c in ctxs}) != len(ctxs):
        raise FriError(FRI_EINVAL, "a context appears twice: pass each context once (depth sets the commits in flight)")
    gen = [c.commit_info()[0] for c in ctxs]     # every enqueued commit bumps its context's generation by one
    out: List[Optional[FRIProof]] = [None] * len(polys)
    pend = []

    def collect(i, j, ticket, g):
        out[i] = _mirror_commit(ctxs[j].commit_wait(ticket), ctxs[j], log_n, channels[i], generation=g)

    try:
        for i, (c, ch) in enumerate(zip(polys, channels)):
            j = i % len(ctxs)
            if len(pend) == depth * len(ctxs):
                collect(*pend.pop(0))
            st = bytes.fromhex(ch.state) if ch.state else None
            t = ctxs[j].commit_async(c, log_n, offset, channel_state=st)
            gen[j] += 1
            pend.append((i, j, t, gen[j]))
        while pend:
            collect(*pend.pop(0))
    finally:
        # a commit that failed (e.g. a coefficient >= p, reported at its wait)
        # must not leave the others' result slots pending on the contexts:
        # wait for every remaining ticket, discarding its result
        for _, j, t, _ in pend:
            try:
                ctxs[j].commit_wait(t)
            except FriError:
                pass
    return out


def fri_commit_sharded(coeffs: Sequence[int], log_n: int, channel: Channel, ctx: Context,
                       offset: int = GENERATOR) -> FRIProof:
    """fri_commit (fri_commit.rs:72-122) over the ranks attached to ``ctx``
    (one process per GPU, every rank passing the same coefficients and
    channel): coset-sharded on the devices, the same transcript on every rank.
    decommit_fri on the returned proof is collective (all ranks, same order)."""
    st = bytes.fromhex(channel.state) if channel.state else None
    res = ctx.commit_sharded(coeffs, log_n, offset, channel_state=st)
    proof = _mirror_commit(res, ctx, log_n, channel)
    proof.sharded = True
    return proof


def _mirror_commit(res: CommitResult, ctx: Context, log_n: int, channel: Channel,
                   generation: Optional[int] = None) -> FRIProof:
    """Append the messages the device commit sent (root hex per layer, beta
    per round, final value) to ``channel`` and take over its state."""
    roots = [bytes(res.roots[k]) for k in range(res.n_layers)]
    betas = [int(res.betas[r]) for r in range(res.n_rounds)]
    for k, root in enumerate(roots):
        channel.proof.append(root.hex().encode())
        channel.compressed_proof.append(root.hex().encode())
        if k < len(betas):
            channel.proof.append(betas[k].to_bytes(8, "big"))
    fv = int(res.final_value).to_bytes(8, "big")
    channel.proof.append(fv)
    channel.compressed_proof.append(fv)
    channel.state = bytes(res.channel_out.digest).hex() if res.channel_out.has_state else ""
    gen = ctx.commit_info()[0] if generation is None else generation
    return FRIProof(ctx, log_n, roots, betas, int(res.final_value), int(res.final_degree), gen)

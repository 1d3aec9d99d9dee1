"""Cluster token server front end: the reference's Netty transport, batching into the engine.

Mirrors (paths relative to sentinel-cluster/sentinel-cluster-server-default/.../cluster/server):
  NettyTransportServer.java:80-100   TCP server, 2-byte length framing, port 18730 by default
  handler/TokenServerHandler.java     ping -> ConnectionManager, FLOW / PARAM_FLOW -> processors,
                                      no processor -> RESPONSE_STATUS_BAD
  processor/FlowRequestProcessor.java, ParamFlowRequestProcessor.java -> TokenService
  connection/ConnectionManager.java   connected count per namespace (AVG_LOCAL thresholds)

Frames are decoded by the C codec (include/sga_wire.h) into one structure-of-arrays batch for
all connections; every `window_us` (or when the batch fills) the batch is decided by the HIP
engine in arrival order -- consecutive FLOW / PARAM_FLOW / PING segments, so the namespace
limiter sees the same order -- and each response frame goes back on its connection.  The
mocked TimeUtil of the tests is `clock` (default: wall-clock milliseconds).
"""
import asyncio
import ctypes as C
import time
from typing import Callable, Dict, List, Optional

import numpy as np

from . import _lib
from ._lib import SgaWireBatch
from .cluster import DefaultTokenService, Engine

WIRE_FLOW, WIRE_PARAM, WIRE_PING, WIRE_BAD, WIRE_DROP = 1, 2, 3, 4, 5
DEFAULT_CLUSTER_SERVER_PORT = 18730  # ClusterConstants.DEFAULT_CLUSTER_SERVER_PORT


def _bind():
    return _lib.load()


class WireBatch:
    """Owns the arrays of one sga_wire_batch."""

    def __init__(self, cap: int = 1 << 16, vcap: int = 1 << 18, ns_cap: int = 1 << 16):
        self.xid = np.zeros(cap, np.int32)
        self.type = np.zeros(cap, np.int8)
        self.kind = np.zeros(cap, np.int8)
        self.flow_id = np.zeros(cap, np.int64)
        self.count = np.zeros(cap, np.int32)
        self.prio = np.zeros(cap, np.uint8)
        self.voff = np.zeros(cap + 1, np.uint32)
        self.values = np.zeros(max(vcap, 1), np.int64)
        self.ns_off = np.zeros(cap, np.uint32)
        self.ns_len = np.zeros(cap, np.uint32)
        self.ns_bytes = np.zeros(max(ns_cap, 1), np.uint8)
        self.s = SgaWireBatch(cap, vcap, 0, 0, *[a.ctypes.data for a in (
            self.xid, self.type, self.kind, self.flow_id, self.count, self.prio, self.voff, self.values,
            self.ns_off, self.ns_len, self.ns_bytes)], ns_cap, 0)

    @property
    def n(self):
        return self.s.n

    def reset(self):
        self.s.n = 0
        self.s.nv = 0
        self.s.ns_used = 0

    def decode(self, buf: bytes):
        """Decodes whole frames from `buf`; returns (frames, consumed bytes)."""
        L = _bind()
        used = C.c_size_t()
        b = np.frombuffer(buf, np.uint8) if buf else np.zeros(1, np.uint8)
        rc = L.sga_wire_decode(b.ctypes.data, len(buf), C.byref(used), C.byref(self.s))
        if rc < 0:
            raise ValueError("frame longer than 1024 bytes (TooLongFrameException)")
        return rc, used.value

    def namespace(self, i: int) -> str:
        o, n = int(self.ns_off[i]), int(self.ns_len[i])
        return bytes(self.ns_bytes[o:o + n]).decode("utf-8", errors="replace")


def decode_sharded(buf: bytes, batches):
    """sga_wire_decode_sharded: FLOW / PARAM_FLOW frames into batches[splitmix64(flowId) mod G] (G = len(batches),
    one engine per GPU), PING and malformed frames into batches[0], each in arrival order, routed inside the
    decode.  Returns (frames, consumed bytes)."""
    L = _bind()
    used = C.c_size_t()
    b = np.frombuffer(buf, np.uint8) if buf else np.zeros(1, np.uint8)
    arr = (SgaWireBatch * len(batches))(*[x.s for x in batches])
    rc = L.sga_wire_decode_sharded(b.ctypes.data, len(buf), C.byref(used), len(batches), arr)
    for x, a in zip(batches, arr):  # the counters came back in the array's copies
        x.s.n, x.s.nv, x.s.ns_used = a.n, a.nv, a.ns_used
    if rc < 0:
        raise ValueError("frame longer than 1024 bytes (TooLongFrameException)")
    return rc, used.value


def encode_responses(xid, type_, kind, status, remaining, wait_ms, ping_count) -> bytes:
    L = _bind()
    n = len(xid)
    arrs = [np.ascontiguousarray(xid, np.int32), np.ascontiguousarray(type_, np.int8),
            np.ascontiguousarray(kind, np.int8), np.ascontiguousarray(status, np.int32),
            np.ascontiguousarray(remaining, np.int32), np.ascontiguousarray(wait_ms, np.int32),
            np.ascontiguousarray(ping_count, np.int32)]
    out = np.zeros(max(16 * n, 1), np.uint8)
    rc = L.sga_wire_encode(*[a.ctypes.data for a in arrs], n, out.ctypes.data, len(out))
    if rc < 0:
        raise RuntimeError(f"encode failed rc={rc}")
    return out[:rc].tobytes()


class ConnectionManager:
    """connection/ConnectionManager.java: namespace -> connected client addresses."""

    def __init__(self):
        self.groups: Dict[str, set] = {}

    def add_connection(self, namespace: str, address: str) -> int:
        g = self.groups.setdefault(namespace, set())
        g.add(address)
        return len(g)

    def remove_connection(self, address: str) -> List[str]:
        changed = []
        for ns, g in self.groups.items():
            if address in g:
                g.discard(address)
                changed.append(ns)
        return changed

    def connected_count(self, namespace: str) -> int:
        return len(self.groups.get(namespace, ()))


class ClusterTokenServer:
    def __init__(self, engine: Engine, host: str = "127.0.0.1", port: int = DEFAULT_CLUSTER_SERVER_PORT,
                 window_us: int = 200, cap: int = 1 << 16, clock: Optional[Callable[[], int]] = None):
        self.engine = engine
        self.svc = DefaultTokenService(engine)
        self.host, self.port = host, port
        self.window = window_us / 1e6
        self.clock = clock or (lambda: int(time.time() * 1000))
        self.batch = WireBatch(cap, vcap=cap * 4, ns_cap=cap * 8)
        self.conn_of: List[int] = []       # per decoded request: connection id
        self.writers: Dict[int, asyncio.StreamWriter] = {}
        self.addr: Dict[int, str] = {}
        self.cm = ConnectionManager()
        self._scheduled = False
        self._server = None
        self._next_conn = 0
        self._lock = asyncio.Lock()

    async def start(self):
        self._server = await asyncio.start_server(self._on_conn, self.host, self.port)
        self.port = self._server.sockets[0].getsockname()[1]
        return self

    async def stop(self):
        if self._server:
            self._server.close()
            await self._server.wait_closed()
        await self.flush()

    async def _on_conn(self, reader: asyncio.StreamReader, writer: asyncio.StreamWriter):
        cid = self._next_conn
        self._next_conn += 1
        peer = writer.get_extra_info("peername")
        self.writers[cid] = writer
        self.addr[cid] = f"{peer[0]}:{peer[1]}" if peer else f"conn{cid}"
        pending = b""
        try:
            while True:
                data = await reader.read(1 << 16)
                if not data:
                    break
                pending += data
                while pending:
                    async with self._lock:
                        before = self.batch.n
                        try:
                            _, used = self.batch.decode(pending)
                        except ValueError:  # TooLongFrameException: the reference drops the channel
                            writer.close()
                            return
                        self.conn_of += [cid] * (self.batch.n - before)
                        # the decoder also stops when the batch's value or namespace buffer is full;
                        # a complete frame left undecoded means such a capacity stop, not a partial frame
                        full = self.batch.n >= self.batch.s.cap or _complete_frame_at(pending, used)
                        # a frame that does not fit even an empty batch (more parameter values or a longer
                        # namespace than the batch buffers hold) can never be decoded: drop the channel,
                        # as for an over-long frame, instead of flushing empty batches forever
                        stuck = full and used == 0 and before == 0 and self.batch.n == 0
                    if stuck:
                        writer.close()
                        return
                    pending = pending[used:]
                    if full:
                        await self.flush()  # drain, then decode the rest
                    elif used == 0:
                        break  # a partial frame waits for more bytes
                self._schedule()
        finally:
            try:
                await self.flush()
            finally:
                self.writers.pop(cid, None)
                for ns in self.cm.remove_connection(self.addr.get(cid, "")):  # channelInactive
                    self.svc_connected(ns)

    def svc_connected(self, ns: str):
        from .cluster import ClusterFlowRuleManager
        ClusterFlowRuleManager(self.engine).set_connected_count(ns, self.cm.connected_count(ns))

    def _schedule(self):
        if not self._scheduled:
            self._scheduled = True
            asyncio.get_running_loop().call_later(self.window, self._fire)

    def _fire(self):
        self._scheduled = False
        fut = asyncio.ensure_future(self.flush())
        fut.add_done_callback(_consume_exception)

    async def flush(self):
        async with self._lock:
            b = self.batch
            n = b.n
            if n == 0:
                return
            kind = b.kind[:n].copy()
            status = np.zeros(n, np.int32)
            remaining = np.zeros(n, np.int32)
            wait = np.zeros(n, np.int32)
            ping = np.zeros(n, np.int32)
            now = self.clock()
            # consecutive segments of one kind, in arrival order
            i = 0
            while i < n:
                k = kind[i]
                j = i + 1
                while j < n and kind[j] == k:
                    j += 1
                if k == WIRE_FLOW:
                    r = self.svc.request_tokens(b.flow_id[i:j], b.count[i:j], b.prio[i:j], np.full(j - i, now))
                    status[i:j], remaining[i:j], wait[i:j] = r["status"], r["remaining"], r["wait_in_ms"]
                elif k == WIRE_PARAM:
                    params = [b.values[b.voff[q]:b.voff[q + 1]].tolist() for q in range(i, j)]
                    r = self.svc.request_param_tokens(b.flow_id[i:j], b.count[i:j], params, np.full(j - i, now))
                    status[i:j], remaining[i:j] = r["status"], r["remaining"]
                elif k == WIRE_PING:
                    for q in range(i, j):
                        ns = b.namespace(q)
                        ping[q] = self.cm.add_connection(ns, self.addr.get(self.conn_of[q], ""))
                        self.svc_connected(ns)
                i = j
            out: Dict[int, List[int]] = {}
            for q in range(n):
                out.setdefault(self.conn_of[q], []).append(q)
            frames = {}
            for cid, qs in out.items():
                idx = np.asarray(qs)
                frames[cid] = encode_responses(b.xid[idx], b.type[idx], kind[idx], status[idx], remaining[idx],
                                               wait[idx], ping[idx])
            b.reset()
            self.conn_of = []
        # one client that reset or closed its connection must not keep the others' responses back:
        # write errors drop that connection only
        for cid, data in frames.items():
            w = self.writers.get(cid)
            if w is None or not data:
                continue
            try:
                if w.is_closing():
                    raise ConnectionResetError("closed")
                w.write(data)
                await w.drain()
            except (ConnectionError, OSError, RuntimeError):
                self.writers.pop(cid, None)
                try:
                    w.close()
                except Exception:  # noqa: BLE001 - already torn down
                    pass


def _complete_frame_at(buf: bytes, at: int) -> bool:
    """True when buf[at:] starts with a whole length-prefixed frame."""
    if len(buf) - at < 2:
        return False
    return len(buf) - at - 2 >= int.from_bytes(buf[at:at + 2], "big")


def _consume_exception(fut: "asyncio.Future") -> None:
    if not fut.cancelled():
        fut.exception()  # retrieved: a failed timed flush is not reported as "never retrieved"


# ---------------------------------------------------------------- client side (tests, tools)
def frame_flow(xid: int, flow_id: int, count: int, prio: Optional[bool]) -> bytes:
    """FlowRequestDataWriter + DefaultRequestEntityWriter + LengthFieldPrepender(2)."""
    body = xid.to_bytes(4, "big", signed=True) + bytes([1]) + flow_id.to_bytes(8, "big", signed=True) + \
        count.to_bytes(4, "big", signed=True) + (b"" if prio is None else bytes([1 if prio else 0]))
    return len(body).to_bytes(2, "big") + body


def frame_ping(xid: int, namespace: str) -> bytes:
    ns = namespace.encode()
    body = xid.to_bytes(4, "big", signed=True) + bytes([0]) + len(ns).to_bytes(4, "big", signed=True) + ns
    return len(body).to_bytes(2, "big") + body


def frame_param(xid: int, flow_id: int, count: int, params) -> bytes:
    """ParamFlowRequestDataWriter: params as (type, value) with ClusterConstants.PARAM_TYPE_*."""
    body = bytearray(xid.to_bytes(4, "big", signed=True) + bytes([2]) + flow_id.to_bytes(8, "big", signed=True)
                     + count.to_bytes(4, "big", signed=True) + len(params).to_bytes(4, "big", signed=True))
    for v in params:
        if isinstance(v, bool):
            body += bytes([6, 1 if v else 0])
        elif isinstance(v, str):
            s = v.encode()
            body += bytes([7]) + len(s).to_bytes(4, "big", signed=True) + s
        elif -(1 << 31) <= v < (1 << 31):
            body += bytes([0]) + v.to_bytes(4, "big", signed=True)
        else:
            body += bytes([1]) + v.to_bytes(8, "big", signed=True)
    return len(body).to_bytes(2, "big") + bytes(body)


def parse_responses(buf: bytes):
    """Response frames -> list of (xid, type, status, data ints)."""
    out, at = [], 0
    while at + 2 <= len(buf):
        n = int.from_bytes(buf[at:at + 2], "big")
        body = buf[at + 2:at + 2 + n]
        at += 2 + n
        xid = int.from_bytes(body[0:4], "big", signed=True)
        typ = body[4]
        st = int.from_bytes(body[5:6], "big", signed=True)
        data = [int.from_bytes(body[k:k + 4], "big", signed=True) for k in range(6, len(body), 4)]
        out.append((xid, typ, st, data))
    return out


def string_key(s: str) -> int:
    return int(_bind().sga_wire_string_key(s.encode(), len(s.encode())))

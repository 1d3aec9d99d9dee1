"""Cluster token wire codec (include/sga_wire.h) on the CPU: the frames
of the reference's Netty transport decoded into engine batches and responses encoded back.
Known answers transcribed from the reference tests
  FlowResponseDataDecoderTest.testDecode   sentinel-cluster-client-default/src/test/java/com/alibaba/csp/sentinel/cluster/client/codec/data/FlowResponseDataDecoderTest.java:28-37
  PingResponseDataWriterTest                sentinel-cluster-server-default/src/test/java/com/alibaba/csp/sentinel/cluster/server/codec/data/PingResponseDataWriterTest.java:31-46
and the decoders' documented behaviour (DefaultRequestEntityDecoder.java:42-63,
FlowRequestDataDecoder.java:35-48, ParamFlowRequestDataDecoder.java:35-91, PingRequestDataDecoder.java:30-41)."""
import numpy as np
import pytest

from sentinel_amd import token_server as ts


def test_response_kats():
    # FlowResponseDataDecoderTest: remaining 12, waitInMs 13 after xid|type|status
    r = ts.encode_responses([7], [1], [ts.WIRE_FLOW], [0], [12], [13], [0])
    assert r == bytes.fromhex("000e") + (7).to_bytes(4, "big") + bytes([1, 0]) + (12).to_bytes(4, "big") + \
        (13).to_bytes(4, "big")
    assert ts.parse_responses(r) == [(7, 1, 0, [12, 13])]
    # PingResponseDataWriterTest: 120 and Integer.MAX_VALUE
    r = ts.encode_responses([1, 2], [0, 0], [ts.WIRE_PING] * 2, [0, 0], [0, 0], [0, 0], [120, 2 ** 31 - 1])
    assert ts.parse_responses(r) == [(1, 0, 0, [120]), (2, 0, 0, [2 ** 31 - 1])]
    # PARAM_FLOW responses carry waitInMs 0 (ParamFlowRequestProcessor), BAD carries no data, DROP nothing
    r = ts.encode_responses([3, 4, 5], [2, 9, 3], [ts.WIRE_PARAM, ts.WIRE_BAD, ts.WIRE_DROP], [1, 0, 0], [0, 0, 0],
                            [50, 0, 0], [0, 0, 0])
    assert ts.parse_responses(r) == [(3, 2, 1, [0, 0]), (4, 9, -1, [])]


def _decode(buf, cap=64):
    b = ts.WireBatch(cap, 256, 1024)
    frames, used = b.decode(buf)
    return b, frames, used


def test_decode_requests():
    buf = (ts.frame_ping(1, "default") + ts.frame_flow(2, 11, 3, True) + ts.frame_flow(3, 12, 1, None) +
           ts.frame_param(4, 5, 2, [3, "a", True, 1 << 40]))
    b, frames, used = _decode(buf)
    assert frames == 4 and used == len(buf)
    assert list(b.kind[:4]) == [ts.WIRE_PING, ts.WIRE_FLOW, ts.WIRE_FLOW, ts.WIRE_PARAM]
    assert list(b.xid[:4]) == [1, 2, 3, 4] and b.namespace(0) == "default"
    assert list(b.flow_id[1:4]) == [11, 12, 5] and list(b.count[1:4]) == [3, 1, 2]
    assert list(b.prio[1:3]) == [1, 0]  # no priority byte -> false
    from sentinel_amd.cluster import param_value_key
    assert list(b.values[b.voff[3]:b.voff[4]]) == [3, param_value_key("a"), 1231, 1 << 40]


def test_decode_malformed_frames():
    head = lambda xid, t: xid.to_bytes(4, "big") + bytes([t])
    fr = lambda body: len(body).to_bytes(2, "big") + body
    cases = [
        (fr(head(1, 0)), ts.WIRE_BAD),                                    # ping without data
        (fr(head(1, 0) + (3).to_bytes(4, "big") + b"  \t"), ts.WIRE_BAD),  # blank namespace
        (fr(head(1, 0) + (9).to_bytes(4, "big") + b"ns"), ts.WIRE_DROP),   # readBytes past the end
        (fr(head(1, 1) + b"\x00" * 11), ts.WIRE_DROP),                     # < 12 data bytes: processor NPE
        (fr(head(1, 3) + b"\x00" * 12), ts.WIRE_DROP),                     # no decoder for type 3
        (fr(head(1, 2) + b"\x00" * 12 + (0).to_bytes(4, "big")), ts.WIRE_DROP),  # amount 0
        (fr(b"\x00\x00\x00"), ts.WIRE_DROP),                               # shorter than xid|type
    ]
    for buf, kind in cases:
        b, frames, _ = _decode(buf)
        assert frames == 1 and b.kind[0] == kind, (buf, b.kind[0])
    # unknown param type is skipped and decoding continues with the next byte
    body = head(9, 2) + (5).to_bytes(8, "big") + (1).to_bytes(4, "big") + (2).to_bytes(4, "big") + bytes([99]) + \
        bytes([0]) + (42).to_bytes(4, "big")
    b, frames, _ = _decode(fr(body))
    assert b.kind[0] == ts.WIRE_PARAM and list(b.values[:b.s.nv]) == [42]


def test_partial_frames_and_limits():
    buf = ts.frame_flow(1, 7, 1, False) * 3
    b, frames, used = _decode(buf[:-3])
    assert frames == 2 and used == 2 * len(ts.frame_flow(1, 7, 1, False))
    frames, used2 = b.decode(buf[used:])   # the rest of the stream continues the same batch
    assert frames == 1 and b.n == 3
    b, frames, used = _decode(buf, cap=2)  # batch full: stops, rest left for the next call
    assert frames == 2 and b.n == 2
    with pytest.raises(ValueError):       # LengthFieldBasedFrameDecoder(1024): TooLongFrameException
        _decode((1025).to_bytes(2, "big") + b"\x00" * 1025)


def test_decode_sharded_equals_decode_then_route():
    """sga_wire_decode_sharded (routing inside the decode): every shard's batch holds exactly
    the FLOW / PARAM_FLOW frames whose flowId maps to it under sga_route_shards' function (splitmix64(flowId)
    mod G), in arrival order, with their values; PING and malformed frames go to shard 0."""
    from sentinel_amd.workload import shard_of
    rng = np.random.default_rng(5)
    frames, meta = [], []
    for x in range(400):
        u = rng.random()
        if u < 0.1:
            frames.append(ts.frame_ping(x, "ns%d" % (x % 3)))
            meta.append(("ping", x, None))
        elif u < 0.6:
            f = int(rng.integers(1, 10_000))
            frames.append(ts.frame_flow(x, f, int(rng.integers(1, 4)), bool(rng.random() < 0.2)))
            meta.append(("flow", x, f))
        else:
            f = int(rng.integers(1, 10_000))
            frames.append(ts.frame_param(x, f, 1, [int(v) for v in rng.integers(0, 50, size=int(rng.integers(1, 4)))]))
            meta.append(("param", x, f))
    buf = b"".join(frames)
    whole = ts.WireBatch(1024, 4096, 4096)
    nf, used = whole.decode(buf)
    assert nf == len(frames) and used == len(buf)
    for G in (1, 2, 8):
        bs = [ts.WireBatch(1024, 4096, 4096) for _ in range(G)]
        nfs, used_s = ts.decode_sharded(buf, bs)
        assert nfs == len(frames) and used_s == len(buf)
        shard = [0 if k == "ping" else int(shard_of(np.array([f], np.int64), G)[0]) for k, _, f in meta]
        for g in range(G):
            idx = [i for i in range(len(meta)) if shard[i] == g]
            b = bs[g]
            assert b.n == len(idx)
            assert list(b.xid[:b.n]) == list(whole.xid[idx]) and list(b.kind[:b.n]) == list(whole.kind[idx])
            assert list(b.flow_id[:b.n]) == list(whole.flow_id[idx]) and list(b.count[:b.n]) == list(whole.count[idx])
            for j, i in enumerate(idx):
                assert list(b.values[b.voff[j]:b.voff[j + 1]]) == list(whole.values[whole.voff[i]:whole.voff[i + 1]])
                if meta[i][0] == "ping":
                    assert b.namespace(j) == whole.namespace(i)

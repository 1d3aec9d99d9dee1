"""End to end through the cluster token wire front end: clients speak
the reference's Netty protocol to ClusterTokenServer (asyncio, batching frames into the HIP
engine); responses are compared with the oracle's replay of the same requests in arrival order
(DefaultTokenService over ClusterFlowChecker / ClusterParamFlowChecker) at the server's mocked
clock.  PING frames drive the connected count of AVG_LOCAL thresholds, as ConnectionManager does."""
import asyncio
import ctypes as C

import numpy as np
import pytest

from tests import oracle_harness as H

pytestmark = pytest.mark.gpu
T0 = 1_700_000_000_000


def _split_frames(buf):
    out, at = [], 0
    while at + 2 <= len(buf):
        n = int.from_bytes(buf[at:at + 2], "big")
        if at + 2 + n > len(buf):
            break
        out.append(buf[at:at + 2 + n])
        at += 2 + n
    return out, buf[at:]


async def _recv(reader, n):
    from sentinel_amd import token_server as ts
    frames, rest = [], b""
    while len(frames) < n:
        rest += await asyncio.wait_for(reader.read(1 << 16), timeout=30)
        f, rest = _split_frames(rest)
        frames += f
    return ts.parse_responses(b"".join(frames))


def test_token_server_end_to_end():
    from sentinel_amd import cluster
    from sentinel_amd import token_server as ts
    rng = np.random.default_rng(5)
    flow_rules = [{"flow_id": f, "count": float(rng.integers(2, 9)), "threshold_type": int(f % 2)} for f in range(1, 21)]
    param_rules = [{"flow_id": f, "count": float(rng.integers(1, 4)), "threshold_type": 1} for f in range(100, 105)]
    eng = cluster.Engine(max_batch=1 << 16)
    cluster.ClusterFlowRuleManager(eng).load_rules("default", [
        cluster.FlowRule(resource=f"r{r['flow_id']}", count=r["count"], cluster_mode=True,
                         cluster_config=cluster.ClusterFlowConfig(flow_id=r["flow_id"],
                                                                  threshold_type=r["threshold_type"]))
        for r in flow_rules])
    cluster.ClusterParamFlowRuleManager(eng).load_rules("default", [
        cluster.ParamFlowRule(resource=f"p{r['flow_id']}", count=r["count"], cluster_mode=True,
                              cluster_config=cluster.ParamFlowClusterConfig(flow_id=r["flow_id"], threshold_type=1))
        for r in param_rules])
    L = H.lib()
    oh = L.orc_cluster_new(1.0, 1.0)
    L.orc_cluster_load_rules(oh, b"default", H.cluster_rules_array(flow_rules), len(flow_rules))
    keep = []
    L.orc_cluster_load_param_rules(oh, b"default", H.cluster_param_rules_array(param_rules, keep), len(param_rules))
    now = [T0]

    # three bursts of requests on connection A, at three clock values
    bursts = []
    xid = 100
    for k in range(3):
        reqs = []
        for _ in range(400):
            xid += 1
            if rng.random() < 0.8:
                reqs.append(("flow", xid, int(rng.integers(1, 23)), int(rng.integers(1, 3)), bool(rng.random() < 0.1)))
            else:
                vals = [int(v) for v in rng.integers(0, 6, size=int(rng.integers(1, 3)))]
                reqs.append(("param", xid, int(rng.integers(99, 106)), 1, vals))
        bursts.append(reqs)

    async def main():
        srv = await ts.ClusterTokenServer(eng, port=0, window_us=500, clock=lambda: now[0]).start()
        ra, wa = await asyncio.open_connection("127.0.0.1", srv.port)
        rb, wb = await asyncio.open_connection("127.0.0.1", srv.port)
        wa.write(ts.frame_ping(1, "default"))
        await wa.drain()
        assert (await _recv(ra, 1)) == [(1, 0, 0, [1])]
        wb.write(ts.frame_ping(2, "default"))
        await wb.drain()
        assert (await _recv(rb, 1)) == [(2, 0, 0, [2])]  # two clients in the namespace
        results = []
        for k, reqs in enumerate(bursts):
            now[0] = T0 + 250 * k
            data = b"".join(ts.frame_flow(x, f, c, p) if kind == "flow" else ts.frame_param(x, f, c, p)
                            for kind, x, f, c, p in reqs)
            wa.write(data)
            await wa.drain()
            results.append(await _recv(ra, len(reqs)))
        wa.close()
        wb.close()
        await srv.stop()
        return results

    results = asyncio.run(main())
    L.orc_cluster_set_connected_count(oh, b"default", 2)
    for k, (reqs, got) in enumerate(zip(bursts, results)):
        t = T0 + 250 * k
        assert [g[0] for g in got] == [r[1] for r in reqs]  # responses in request order
        for (kind, x, f, c, p), (gx, gtype, gst, gdata) in zip(reqs, got):
            if kind == "flow":
                o = L.orc_cluster_request_token(oh, f, c, 1 if p else 0, t)
                assert (gtype, gst, gdata) == (1, o.status, [o.remaining, o.wait_in_ms]), (k, x, f, c, p)
            else:
                vals = (C.c_int64 * len(p))(*[cluster.param_value_key(v) for v in p])
                o = L.orc_cluster_request_param_token(oh, f, c, vals, len(p), t)
                assert (gtype, gst, gdata) == (2, o.status, [o.remaining, 0]), (k, x, f, c, p)
    L.orc_cluster_free(oh)
    eng.close()

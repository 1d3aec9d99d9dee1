package com.alibaba.csp.sentinel.gpu;

import java.util.Collection;
import java.util.Map;
import java.util.concurrent.ConcurrentHashMap;
import java.util.concurrent.atomic.AtomicInteger;

import com.alibaba.csp.sentinel.cluster.TokenResult;
import com.alibaba.csp.sentinel.cluster.TokenResultStatus;
import com.alibaba.csp.sentinel.cluster.TokenService;
import com.alibaba.csp.sentinel.spi.Spi;
import com.alibaba.csp.sentinel.util.TimeUtil;

/**
 * {@link TokenService} (sentinel-core/.../cluster/TokenService.java:26-62) decided by the MI355X engine.
 * Registered in META-INF/services/com.alibaba.csp.sentinel.cluster.TokenService ahead of
 * DefaultTokenService, so TokenServiceProvider (sentinel-cluster-server-default/.../TokenServiceProvider.java:38-45)
 * resolves it and FlowRequestProcessor / the embedded server call it unchanged.  Each call is one
 * request; the engine's coalescing queue (sga_request_token_one) gathers concurrent callers -- one per
 * Netty worker -- into one launch.
 */
@Spi(order = -100)
public class GpuTokenService implements TokenService {

    private final long engine = GpuEngine.get();
    private final Map<String, Integer> clientIds = new ConcurrentHashMap<>();
    private final AtomicInteger nextClientId = new AtomicInteger();

    private static TokenResult result(int rc, int[] o) {
        if (rc != GpuEngine.OK) {
            return new TokenResult(TokenResultStatus.FAIL);
        }
        return new TokenResult(o[0]).setRemaining(o[1]).setWaitInMs(o[2]);
    }

    @Override
    public TokenResult requestToken(Long ruleId, int acquireCount, boolean prioritized) {
        if (ruleId == null) {  // DefaultTokenService.notValidRequest -> BAD_REQUEST (the engine checks it too)
            return new TokenResult(TokenResultStatus.BAD_REQUEST);
        }
        int[] o = new int[3];
        int rc = GpuEngine.requestToken(engine, ruleId, acquireCount, prioritized, TimeUtil.currentTimeMillis(), o);
        return result(rc, o);
    }

    @Override
    public TokenResult requestParamToken(Long ruleId, int acquireCount, Collection<Object> params) {
        if (ruleId == null || params == null || params.isEmpty()) {
            return new TokenResult(TokenResultStatus.BAD_REQUEST);
        }
        long[] keys = new long[params.size()];
        int i = 0;
        for (Object p : params) {
            keys[i++] = GpuArgs.key(p);
        }
        int[] o = new int[3];
        int rc = GpuEngine.requestParamToken(engine, ruleId, acquireCount, keys, TimeUtil.currentTimeMillis(), o);
        return result(rc, o);
    }

    @Override
    public TokenResult requestConcurrentToken(String clientAddress, Long ruleId, int acquireCount) {
        if (clientAddress == null || ruleId == null) {
            return new TokenResult(TokenResultStatus.BAD_REQUEST);
        }
        long[] o = new long[2];
        int rc = GpuEngine.concurrent(engine, 0, clientId(clientAddress), ruleId, acquireCount,
                                      TimeUtil.currentTimeMillis(), o);
        if (rc != GpuEngine.OK) {
            return new TokenResult(TokenResultStatus.FAIL);
        }
        TokenResult r = new TokenResult((int) o[0]);
        r.setTokenId(o[1]);
        return r;
    }

    @Override
    public void releaseConcurrentToken(Long tokenId) {
        if (tokenId == null) {
            return;
        }
        GpuEngine.concurrent(engine, 1, 0, tokenId, 0, TimeUtil.currentTimeMillis(), new long[2]);
    }

    private int clientId(String address) {  // dense, unique per address (an AtomicInteger, not size())
        return clientIds.computeIfAbsent(address, a -> nextClientId.getAndIncrement());
    }
}

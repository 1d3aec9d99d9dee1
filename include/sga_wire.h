/*
 * sga_wire.h -- the Sentinel cluster token protocol (the Netty transport of the default token
 * server) decoded into engine batches and encoded back.  Part of libsentinel_amd.so.
 *
 * Reference framing and entities (paths relative to
 * sentinel-cluster/sentinel-cluster-server-default/src/main/java/com/alibaba/csp/sentinel/cluster/server):
 *   frame            LengthFieldBasedFrameDecoder(1024, 0, 2, 0, 2) / LengthFieldPrepender(2)
 *                    NettyTransportServer.java:89-91  (u16 big-endian length, body <= 1024 bytes)
 *   request          xid i32 | type i8 | data          codec/DefaultRequestEntityDecoder.java:42-63
 *     PING (0)       len i32 | namespace bytes         codec/data/PingRequestDataDecoder.java:30-41
 *     FLOW (1)       flowId i64 | count i32 [| prio bool]   codec/data/FlowRequestDataDecoder.java:35-48
 *     PARAM_FLOW (2) flowId i64 | count i32 | n i32 | n typed params
 *                                                      codec/data/ParamFlowRequestDataDecoder.java:35-91
 *   response         xid i32 | type i8 | status i8 | data   codec/DefaultResponseEntityWriter.java:35-52
 *     FLOW / PARAM   remaining i32 | waitInMs i32      codec/data/FlowResponseDataWriter.java:30-34
 *     PING           connected count i32               codec/data/PingResponseDataWriter.java:30-35
 * Constants: sentinel-cluster-common-default/.../cluster/ClusterConstants.java:22-47.
 * All multi-byte fields are big endian (Netty ByteBuf).
 */
#ifndef SGA_WIRE_H
#define SGA_WIRE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SGA_MSG_PING 0
#define SGA_MSG_FLOW 1
#define SGA_MSG_PARAM_FLOW 2
#define SGA_MSG_CONCURRENT_ACQUIRE 3
#define SGA_MSG_CONCURRENT_RELEASE 4

#define SGA_WIRE_MAX_FRAME 1024 /* LengthFieldBasedFrameDecoder maxFrameLength */

/* Request kinds after decoding (what the server does with the frame). */
#define SGA_WIRE_FLOW 1        /* -> TokenService.requestToken */
#define SGA_WIRE_PARAM 2       /* -> TokenService.requestParamToken */
#define SGA_WIRE_PING 3        /* -> ConnectionManager.addConnection(namespace) */
#define SGA_WIRE_BAD 4         /* no processor / undecodable data: RESPONSE_STATUS_BAD (-1) */
#define SGA_WIRE_DROP 5        /* DefaultRequestEntityDecoder returned null: no response */

/* Decoded requests, structure of arrays, capacity `cap` requests / `vcap` parameter values. */
typedef struct sga_wire_batch {
    size_t cap, vcap;
    size_t n, nv;        /* decoded requests / values */
    int32_t *xid;
    int8_t *type;        /* message type byte as received */
    int8_t *kind;        /* SGA_WIRE_* */
    int64_t *flow_id;
    int32_t *count;
    uint8_t *prio;
    uint32_t *voff;      /* n + 1 offsets into values (PARAM requests; others contribute 0) */
    int64_t *values;     /* parameter keys (sga_wire_param_key) */
    uint32_t *ns_off;    /* PING: namespace bytes at ns_bytes[ns_off[i] .. ns_off[i] + ns_len[i]) */
    uint32_t *ns_len;
    uint8_t *ns_bytes;
    size_t ns_cap, ns_used;
} sga_wire_batch;

/* 64-bit key of a typed parameter (the engine's stand-in for the Java Object):
 *   INTEGER/LONG/SHORT/BYTE -> the value; BOOLEAN -> Boolean.hashCode (1231 / 1237);
 *   DOUBLE / FLOAT -> IEEE bits; STRING -> FNV-1a 64 of the bytes.
 * Distinct Objects with equal keys (e.g. Integer 5 and Long 5 for one rule) share a counter. */
int64_t sga_wire_string_key(const uint8_t *bytes, size_t len);

/* Decodes as many whole frames as `buf` holds; *consumed = bytes used (a partial frame at the end
 * is left for the next call).  Stops early when the batch is full.  Returns the number of frames
 * decoded, or -EINVAL for a frame longer than SGA_WIRE_MAX_FRAME (the reference closes such a
 * connection: TooLongFrameException). */
int sga_wire_decode(const uint8_t *buf, size_t len, size_t *consumed, sga_wire_batch *out);

/* sga_wire_decode into G per-shard batches (the multi-GPU token server, one engine per GPU): a FLOW /
 * PARAM_FLOW frame goes to outs[splitmix64(flowId) mod G] -- the shard function of sga_route_shards --,
 * PING and malformed frames to outs[0]; each batch keeps arrival order.  The routing happens inside the
 * decode (no separate pass over the requests).  Stops when the batch a frame goes to is full. */
int sga_wire_decode_sharded(const uint8_t *buf, size_t len, size_t *consumed, uint32_t G, sga_wire_batch *outs);

/* Encodes one response frame per request i in [0, n): FLOW / PARAM from token results
 * (status = TokenResultStatus, remaining, waitInMs; PARAM responses carry waitInMs 0,
 * ParamFlowRequestProcessor.java:48-54), PING with `ping_count[i]`, BAD as status -1 without data,
 * DROP as nothing.  Writes at most `cap` bytes; returns bytes written or -ERANGE. */
int sga_wire_encode(const int32_t *xid, const int8_t *type, const int8_t *kind, const int32_t *status,
                    const int32_t *remaining, const int32_t *wait_ms, const int32_t *ping_count, size_t n,
                    uint8_t *out, size_t cap);

#ifdef __cplusplus
}
#endif
#endif

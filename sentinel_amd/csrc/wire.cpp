// Sentinel cluster token protocol <-> engine batches (include/sga_wire.h).  Host code: the frames
// arrive on sockets; the decoded structure-of-arrays batch is what sga_request_tokens /
// sga_request_param_tokens take, so one decode call turns many connections' frames into one
// engine launch.
#include "../../include/sga_wire.h"
#include "common.hpp"  // splitmix64 (the shard function of sga_route_shards)

#include <cerrno>
#include <cstring>

namespace {

struct Reader {
    const uint8_t *p;
    size_t n, at = 0;
    bool ok = true;
    size_t left() const { return n - at; }
    uint64_t be(int bytes) {
        if (at + bytes > n) {  // ByteBuf.readXxx past the end: IndexOutOfBoundsException
            ok = false;
            at = n;
            return 0;
        }
        uint64_t v = 0;
        for (int i = 0; i < bytes; ++i) v = (v << 8) | p[at + i];
        at += bytes;
        return v;
    }
    int8_t i8() { return (int8_t)be(1); }
    int16_t i16() { return (int16_t)be(2); }
    int32_t i32() { return (int32_t)be(4); }
    int64_t i64() { return (int64_t)be(8); }
};

enum : int { P_INTEGER = 0, P_LONG, P_BYTE, P_DOUBLE, P_FLOAT, P_SHORT, P_BOOLEAN, P_STRING };

}  // namespace

extern "C" {

int64_t sga_wire_string_key(const uint8_t *b, size_t len) {
    uint64_t h = 0xcbf29ce484222325ULL;  // FNV-1a 64
    for (size_t i = 0; i < len; ++i) {
        h ^= b[i];
        h *= 0x100000001b3ULL;
    }
    return (int64_t)h;
}

}  // extern "C"

namespace {

void batch_begin(sga_wire_batch *o) {  // a batch's first decode call
    if (o->n == 0) {
        o->nv = 0;
        o->ns_used = 0;
        if (o->voff) o->voff[0] = 0;
    }
}

// The frame loop of sga_wire_decode / sga_wire_decode_sharded: pick(frame, flen) names the batch a frame goes
// to (from the frame's first bytes), the rest is one decoder.
template <bool kPrefetch, class Pick>
int decode_frames(const uint8_t *buf, size_t len, size_t *consumed, Pick pick) {
    size_t at = 0;
    int frames = 0;
    while (len - at >= 2) {
        const size_t flen = ((size_t)buf[at] << 8) | buf[at + 1];
        if (flen > SGA_WIRE_MAX_FRAME) {
            *consumed = at;
            return -EINVAL;
        }
        if (len - at - 2 < flen) break;  // partial frame
        sga_wire_batch *o = pick(buf + at + 2, flen);
        if (o->n >= o->cap) break;
        Reader r{buf + at + 2, flen};
        const size_t i = o->n;
        if (kPrefetch) {  // G interleaved output streams per array outrun the hardware prefetchers
            if ((i & 7) == 0) {
                __builtin_prefetch(o->flow_id + i + 64, 1);
                __builtin_prefetch(o->xid + i + 64, 1);
                __builtin_prefetch(o->count + i + 64, 1);
                __builtin_prefetch(o->ns_off + i + 64, 1);
                __builtin_prefetch(o->ns_len + i + 64, 1);
                __builtin_prefetch(o->voff + i + 65, 1);
            }
            if ((i & 63) == 0) {
                __builtin_prefetch(o->type + i + 256, 1);
                __builtin_prefetch(o->kind + i + 256, 1);
                __builtin_prefetch(o->prio + i + 256, 1);
            }
        }
        int8_t kind = SGA_WIRE_DROP;
        int32_t xid = 0;
        int8_t type = 0;
        int64_t fid = 0;
        int32_t cnt = 0;
        uint8_t prio = 0;
        const size_t v0 = o->nv, ns0 = o->ns_used;
        uint32_t nsl = 0;
        bool full = false;
        // DefaultRequestEntityDecoder.decode, :42-63
        if (r.left() >= 5) {
            xid = r.i32();
            type = r.i8();
            const bool has_data = r.left() > 0;
            if (type == SGA_MSG_PING) {
                // PingRequestDataDecoder: length i32, then that many bytes (length > 0)
                kind = SGA_WIRE_BAD;  // TokenServerHandler.handlePingRequest: null / blank namespace
                if (has_data && r.left() >= 4) {
                    const int32_t l = r.i32();
                    if (l > 0 && r.left() > 0) {
                        if ((size_t)l > r.left()) {
                            kind = SGA_WIRE_DROP;  // readBytes past the end
                        } else if (o->ns_used + (size_t)l > o->ns_cap) {
                            full = true;
                        } else {
                            bool blank = true;  // StringUtil.isBlank
                            for (int32_t k = 0; k < l; ++k) {
                                const uint8_t c = r.p[r.at + k];
                                if (!(c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == 0x0B))
                                    blank = false;
                            }
                            std::memcpy(o->ns_bytes + o->ns_used, r.p + r.at, (size_t)l);
                            nsl = (uint32_t)l;
                            o->ns_used += (size_t)l;
                            r.at += (size_t)l;
                            kind = blank ? SGA_WIRE_BAD : SGA_WIRE_PING;
                        }
                    }
                }
            } else if (type == SGA_MSG_FLOW) {
                // FlowRequestDataDecoder: >= 12 bytes, prio when one more byte is there; a null data
                // object makes FlowRequestProcessor throw (no response)
                if (has_data && r.left() >= 12) {
                    fid = r.i64();
                    cnt = r.i32();
                    if (r.left() >= 1) prio = r.i8() != 0;
                    kind = SGA_WIRE_FLOW;
                }
            } else if (type == SGA_MSG_PARAM_FLOW) {
                // ParamFlowRequestDataDecoder: >= 16 bytes, amount > 0 typed params
                if (has_data && r.left() >= 16) {
                    fid = r.i64();
                    cnt = r.i32();
                    const int32_t amount = r.i32();
                    if (amount > 0) {
                        for (int32_t k = 0; k < amount && r.ok; ++k) {
                            const int8_t pt = r.i8();
                            int64_t key = 0;
                            bool add = true;
                            switch (pt) {
                            case P_INTEGER: key = r.i32(); break;
                            case P_STRING: {
                                const int32_t l = r.i32();
                                if (l < 0 || (size_t)l > r.left()) {
                                    r.ok = false;  // NegativeArraySize / IndexOutOfBounds
                                    break;
                                }
                                key = sga_wire_string_key(r.p + r.at, (size_t)l);
                                r.at += (size_t)l;
                                break;
                            }
                            case P_BOOLEAN: key = r.i8() != 0 ? 1231 : 1237; break;
                            case P_DOUBLE: key = r.i64(); break;
                            case P_LONG: key = r.i64(); break;
                            case P_FLOAT: key = (int64_t)(uint32_t)r.i32(); break;
                            case P_BYTE: key = r.i8(); break;
                            case P_SHORT: key = r.i16(); break;
                            default: add = false;  // unknown type: skipped, decoding continues
                            }
                            if (!r.ok) break;
                            if (add) {
                                if (o->nv >= o->vcap) {
                                    full = true;
                                    break;
                                }
                                o->values[o->nv++] = key;
                            }
                        }
                        if (r.ok) kind = SGA_WIRE_PARAM;
                    }
                }
            } else {
                kind = SGA_WIRE_DROP;  // no decoder registered: the decoder returns null
            }
        }
        if (full) {  // undo this frame and stop: the caller drains the batch and calls again
            o->nv = v0;
            o->ns_used = ns0;
            break;
        }
        if (kind != SGA_WIRE_PARAM) o->nv = v0;
        if (kind != SGA_WIRE_PING) {
            o->ns_used = ns0;
            nsl = 0;
        }
        o->xid[i] = xid;
        o->type[i] = type;
        o->kind[i] = kind;
        o->flow_id[i] = fid;
        o->count[i] = cnt;
        o->prio[i] = prio;
        o->ns_off[i] = (uint32_t)ns0;
        o->ns_len[i] = nsl;
        o->voff[i + 1] = (uint32_t)o->nv;
        o->n = i + 1;
        at += 2 + flen;
        ++frames;
    }
    *consumed = at;
    return frames;
}

}  // namespace

extern "C" {

int sga_wire_decode(const uint8_t *buf, size_t len, size_t *consumed, sga_wire_batch *o) {
    if (!buf || !consumed || !o) return -EINVAL;
    batch_begin(o);
    return decode_frames<false>(buf, len, consumed, [o](const uint8_t *, size_t) { return o; });
}

// Routing inside the decode (the multi-GPU token server): a FLOW / PARAM_FLOW frame goes to the
// batch of shard splitmix64(flowId) mod G -- the flowId sits right after xid and type, so it is read before
// anything of the frame is stored -- everything else (PING, malformed frames) to batch 0.  Each shard's batch
// keeps arrival order, as sga_route_shards does; no separate pass over the decoded requests.
int sga_wire_decode_sharded(const uint8_t *buf, size_t len, size_t *consumed, uint32_t G, sga_wire_batch *outs) {
    if (!buf || !consumed || !outs || G == 0) return -EINVAL;
    for (uint32_t g = 0; g < G; ++g) batch_begin(&outs[g]);
    const uint64_t mask = (G & (G - 1)) == 0 ? G - 1 : 0;  // a power-of-two G: the modulo is a mask
    return decode_frames<true>(buf, len, consumed, [outs, G, mask](const uint8_t *f, size_t flen) {
        if (flen >= 13 && (f[4] == SGA_MSG_FLOW || f[4] == SGA_MSG_PARAM_FLOW)) {
            uint64_t fid;
            std::memcpy(&fid, f + 5, 8);
            const uint64_t h = sga::splitmix64(__builtin_bswap64(fid));
            return &outs[mask || G == 1 ? h & mask : h % G];
        }
        return &outs[0];
    });
}

int sga_wire_encode(const int32_t *xid, const int8_t *type, const int8_t *kind, const int32_t *status,
                    const int32_t *remaining, const int32_t *wait_ms, const int32_t *ping_count, size_t n,
                    uint8_t *out, size_t cap) {
    if (n && (!xid || !type || !kind || !out)) return -EINVAL;
    size_t at = 0;
    auto put = [&](uint64_t v, int bytes) {
        for (int i = bytes - 1; i >= 0; --i) out[at++] = (uint8_t)(v >> (8 * i));
    };
    for (size_t i = 0; i < n; ++i) {
        size_t body;
        switch (kind[i]) {
        case SGA_WIRE_FLOW:
        case SGA_WIRE_PARAM: body = 6 + 8; break;
        case SGA_WIRE_PING: body = 6 + 4; break;
        case SGA_WIRE_BAD: body = 6; break;
        default: continue;  // no response
        }
        if (at + 2 + body > cap) return -ERANGE;
        put(body, 2);  // LengthFieldPrepender(2)
        put((uint32_t)xid[i], 4);
        put((uint8_t)type[i], 1);
        if (kind[i] == SGA_WIRE_BAD) {
            put((uint8_t)(int8_t)-1, 1);  // ClusterConstants.RESPONSE_STATUS_BAD
        } else if (kind[i] == SGA_WIRE_PING) {
            put(0, 1);  // RESPONSE_STATUS_OK, PingResponseDataWriter: connected count
            put((uint32_t)(ping_count ? ping_count[i] : 0), 4);
        } else {
            put((uint8_t)(int8_t)(status ? status[i] : 0), 1);
            put((uint32_t)(remaining ? remaining[i] : 0), 4);
            put((uint32_t)(kind[i] == SGA_WIRE_PARAM ? 0 : (wait_ms ? wait_ms[i] : 0)), 4);
        }
    }
    return (int)at;
}

}  // extern "C"

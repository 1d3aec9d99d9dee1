"""Java helpers needed host-side (key -> flowId for the Envoy RLS front end)."""


def string_hash_code(s: str) -> int:
    """java.lang.String.hashCode over UTF-16 code units (i32 wrap)."""
    h = 0
    data = s.encode("utf-16-le")
    for i in range(0, len(data), 2):
        cu = data[i] | (data[i + 1] << 8)
        h = (h * 31 + cu) & 0xFFFFFFFF
    return h - (1 << 32) if h >= (1 << 31) else h


def is_blank(s) -> bool:
    """StringUtil.isBlank: null, empty or only Character.isWhitespace chars (sentinel-core util/StringUtil.java:43-54)."""
    if not s:
        return True
    return all(c in " \t\n\x0b\f\r\x1c\x1d\x1e\x1f" or (c.isspace() and c not in "\x85\xa0\u2007\u202f")
               for c in s)


def rls_key(domain: str, entries) -> str:
    """SentinelEnvoyRlsServiceImpl.generateKey: domain|k|v|k|v (RLS/SentinelEnvoyRlsServiceImpl.java:127-133)."""
    parts = [domain]
    for k, v in entries:
        parts.append(k)
        parts.append(v)
    return "|".join(parts)

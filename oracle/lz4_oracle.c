/*
 * lz4_oracle.c — TEST INFRASTRUCTURE ONLY (see lz4_oracle.h).
 *
 * A scalar C restatement of the reference path. It is deliberately written as a
 * straight transcription of the algorithm each function cites, not for speed
 * (bench.py times it as the "port" CPU baseline, compiled -O3 -march=native).
 */
#include "lz4_oracle.h"

#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ xxh32 */
/* twox-hash 2.1.2 XxHash32 (Cargo.toml:43) is the standard XXH32 algorithm. */
#define P1 2654435761U
#define P2 2246822519U
#define P3 3266489917U
#define P4 668265263U
#define P5 374761393U

static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static inline uint32_t rd32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline uint64_t rd64(const uint8_t* p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }
static inline void wr32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}
static inline uint32_t xxh_round(uint32_t acc, uint32_t in) {
    acc += in * P2;
    acc = rotl32(acc, 13);
    return acc * P1;
}

uint32_t or_xxh32(const uint8_t* p, size_t n, uint32_t seed) {
    const uint8_t* end = p + n;
    uint32_t h;
    if (n >= 16) {
        const uint8_t* limit = end - 16;
        uint32_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        do {
            v1 = xxh_round(v1, rd32(p));
            v2 = xxh_round(v2, rd32(p + 4));
            v3 = xxh_round(v3, rd32(p + 8));
            v4 = xxh_round(v4, rd32(p + 12));
            p += 16;
        } while (p <= limit);
        h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
    } else {
        h = seed + P5;
    }
    h += (uint32_t)n;
    while (p + 4 <= end) {
        h += rd32(p) * P3;
        h = rotl32(h, 17) * P4;
        p += 4;
    }
    while (p < end) {
        h += (*p) * P5;
        h = rotl32(h, 11) * P1;
        p++;
    }
    h ^= h >> 15;
    h *= P2;
    h ^= h >> 13;
    h *= P3;
    h ^= h >> 16;
    return h;
}

/* ------------------------------------------------------------- constants */
#define LZ4F_MAGIC 0x184D2204u
#define LZ4F_LEGACY_MAGIC 0x184C2102u
#define STORE_MODE_MAX_BLOCK (4u * 1024u * 1024u) /* compression.rs:42 */
#define BLOCK_UNCOMPRESSED_BIT 0x80000000u        /* compression.rs:47 */
#define FLG_VERSION_MASK 0xC0u
#define FLG_VERSION_01 0x40u
#define FLG_INDEPENDENT 0x20u
#define FLG_BLOCK_CHECKSUM 0x10u
#define FLG_CONTENT_SIZE 0x08u
#define FLG_CONTENT_CHECKSUM 0x04u
#define FLG_RESERVED 0x02u
#define FLG_DICT_ID 0x01u
#define BD_RESERVED 0x8Fu

/* lz4_flex block constants. */
#define MINMATCH 4
#define MFLIMIT 12
#define LAST_LITERALS 5
#define END_OFFSET (LAST_LITERALS + 1)
#define LZ4_MIN_LENGTH (MFLIMIT + 1)
#define MAX_DISTANCE 65535u

static size_t block_size_of_code(unsigned code) {
    switch (code) {
        case 4: return 64u * 1024u;
        case 5: return 256u * 1024u;
        case 6: return 1024u * 1024u;
        case 7: return 4u * 1024u * 1024u;
        default: return 0;
    }
}

size_t or_frame_bound(size_t n) {
    /* Worst case over every frame shape written here: 64 KiB blocks, each stored
     * (4-byte word + raw bytes), plus header (7), end mark (4), checksum (4). */
    size_t blocks = n / (64u * 1024u) + 1;
    return n + 4 * blocks + 15;
}

/* -------------------------------------------------- store mode (a3) */
/* compression.rs:326-368, byte for byte. */
int or_store_mode_frame(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len) {
    size_t blocks = (n + STORE_MODE_MAX_BLOCK - 1) / STORE_MODE_MAX_BLOCK; /* data.chunks(4 MiB) */
    size_t need = n + 4 * blocks + 15;
    if (cap < need) return OR_DST_TOO_SMALL;
    uint8_t* o = dst;
    const uint8_t flg = FLG_VERSION_01 | FLG_INDEPENDENT | FLG_CONTENT_CHECKSUM; /* :329-334 */
    const uint8_t bd = 7u << 4;                                                   /* :335 */
    uint8_t fd[2] = {flg, bd};
    wr32(o, LZ4F_MAGIC); o += 4;
    *o++ = flg;
    *o++ = bd;
    *o++ = (uint8_t)(or_xxh32(fd, 2, 0) >> 8); /* :340-342 */
    for (size_t off = 0; off < n; off += STORE_MODE_MAX_BLOCK) {
        size_t len = n - off < STORE_MODE_MAX_BLOCK ? n - off : STORE_MODE_MAX_BLOCK;
        wr32(o, (uint32_t)len | BLOCK_UNCOMPRESSED_BIT); o += 4; /* :355 */
        memcpy(o, src + off, len); o += len;
    }
    wr32(o, 0); o += 4;                    /* :361 end mark */
    wr32(o, or_xxh32(src, n, 0)); o += 4;  /* :364-365 content checksum */
    *out_len = (size_t)(o - dst);
    return OR_OK;
}

/* ------------------------------------- lz4_flex block compressor (a1) */
/* Restated from lz4_flex 0.11 block/compress.rs compress_internal as used by
 * frame/compress.rs FrameEncoder::write_block (HashTable4K: 4096 x u32 entries,
 * 5-byte hash on 64-bit targets; table persists across the frame's blocks and
 * stale entries below the stream offset are skipped).
 *
 * Hash choice (SURVEY.md A.3 erratum): the size-dependent table selection
 * (input < u16::MAX -> HashTable4KU16 with the 4-byte hash) belongs to the BLOCK API
 * (compress_into / compress_into_sink_with_dict). The frame encoder owns one HashTable4K
 * field for its whole life and calls compress_internal directly: its entries are
 * pos + input_stream_offset, which a u16 table cannot hold past the first 64 KiB of a
 * stream, so the frame path uses the u32 table for every input size, and that table's
 * get_hash_at is hash5 on 64-bit targets. Recalled (the crate is absent): unpinned. */
typedef struct { uint32_t t[4096]; } ht4k_t;

static inline uint32_t hash5_idx(const uint8_t* in, size_t pos) {
    uint64_t seq = rd64(in + pos);
    uint64_t h = ((seq << 24) * 889523592379ULL) >> 48; /* hash5 */
    return (uint32_t)(h >> 4);                          /* HASHTABLE_BIT_SHIFT_4K */
}

typedef struct { uint8_t* p; uint8_t* end; int overflow; } sink_t;
static inline void sink_byte(sink_t* s, uint8_t b) {
    if (s->p < s->end) *s->p++ = b; else s->overflow = 1;
}
static inline void sink_bytes(sink_t* s, const uint8_t* src, size_t n) {
    if ((size_t)(s->end - s->p) >= n) { memcpy(s->p, src, n); s->p += n; } else s->overflow = 1;
}
static inline void write_integer(sink_t* s, size_t n) {
    while (n >= 0xFF) { sink_byte(s, 0xFF); n -= 0xFF; }
    sink_byte(s, (uint8_t)n);
}
static void handle_last_literals(sink_t* s, const uint8_t* input, size_t len, size_t start) {
    size_t lit = len - start;
    sink_byte(s, lit < 0xF ? (uint8_t)(lit << 4) : 0xF0);
    if (lit >= 0xF) write_integer(s, lit - 0xF);
    sink_bytes(s, input + start, lit);
}
/* count_same_bytes: equal bytes from (cur, cand) with cur bounded by len - END_OFFSET. */
static size_t count_same_bytes(const uint8_t* in, size_t cur, size_t cand, size_t cur_end) {
    size_t n = 0;
    while (cur + n < cur_end && in[cur + n] == in[cand + n]) n++;
    return n;
}

static size_t lzf_compress_internal(const uint8_t* input, size_t len, ht4k_t* dict,
                                    size_t stream_off, sink_t* s) {
    uint8_t* start = s->p;
    if (len < LZ4_MIN_LENGTH) {
        handle_last_literals(s, input, len, 0);
        return (size_t)(s->p - start);
    }
    const size_t end_pos_check = len - MFLIMIT;
    size_t literal_start = 0, cur = 0;
    if (stream_off == 0) {
        /* "we can't start with a match": insert position 0, begin at 1 */
        dict->t[hash5_idx(input, 0)] = 0;
        cur = 1;
    }
    for (;;) {
        size_t non_match_count = 1u << 5; /* INCREASE_STEPSIZE_BITSHIFT */
        size_t next_cur = cur;
        size_t cand = 0, offset = 0;
        for (;;) {
            size_t step = non_match_count >> 5;
            non_match_count++;
            cur = next_cur;
            next_cur += step;
            if (cur > end_pos_check) {
                handle_last_literals(s, input, len, literal_start);
                return (size_t)(s->p - start);
            }
            uint32_t h = hash5_idx(input, cur);
            cand = dict->t[h];
            dict->t[h] = (uint32_t)(cur + stream_off);
            if (stream_off + cur - cand > MAX_DISTANCE) continue;
            if (cand < stream_off) continue; /* stale entry from an earlier independent block */
            offset = stream_off + cur - cand;
            cand -= stream_off;
            if (rd32(input + cand) == rd32(input + cur)) break;
        }
        /* backtrack_match */
        while (cand > 0 && cur > literal_start && input[cur - 1] == input[cand - 1]) {
            cur--;
            cand--;
        }
        size_t lit_len = cur - literal_start;
        cur += MINMATCH;
        cand += MINMATCH;
        size_t dup = count_same_bytes(input, cur, cand, len - END_OFFSET);
        cur += dup;
        dict->t[hash5_idx(input, cur - 2)] = (uint32_t)(cur - 2 + stream_off);

        uint8_t token = (uint8_t)((lit_len < 0xF ? lit_len : 0xF) << 4);
        token |= (uint8_t)(dup < 0xF ? dup : 0xF);
        sink_byte(s, token);
        if (lit_len >= 0xF) write_integer(s, lit_len - 0xF);
        sink_bytes(s, input + literal_start, lit_len);
        sink_byte(s, (uint8_t)offset);
        sink_byte(s, (uint8_t)(offset >> 8));
        if (dup >= 0xF) write_integer(s, dup - 0xF);
        literal_start = cur;
    }
}

size_t or_lz4flex_compress_block(const uint8_t* src, size_t n, uint8_t* dst, size_t cap) {
    ht4k_t* ht = (ht4k_t*)calloc(1, sizeof(ht4k_t));
    sink_t s = {dst, dst + cap, 0};
    size_t r = lzf_compress_internal(src, n, ht, 0, &s);
    free(ht);
    return s.overflow ? (size_t)-1 : r;
}

/* FrameEncoder::with_frame_info(FrameInfo{content_checksum, Independent}) + write_all + finish. */
int or_lz4flex_compress_frame(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len) {
    /* BlockSize::from_buf_length on the first (whole-buffer) write; an empty write never
     * opens a frame and finish() opens one with length 0 -> Max64KB. */
    unsigned code = n <= 64u * 1024u ? 4u : (n <= 256u * 1024u ? 5u : 7u);
    size_t bmax = block_size_of_code(code);
    size_t blocks = n == 0 ? 0 : (n + bmax - 1) / bmax;
    if (cap < n + 4 * blocks + 15) return OR_DST_TOO_SMALL;
    uint8_t* o = dst;
    uint8_t flg = FLG_VERSION_01 | FLG_INDEPENDENT | FLG_CONTENT_CHECKSUM;
    uint8_t bd = (uint8_t)(code << 4);
    uint8_t fd[2] = {flg, bd};
    wr32(o, LZ4F_MAGIC); o += 4;
    *o++ = flg;
    *o++ = bd;
    *o++ = (uint8_t)(or_xxh32(fd, 2, 0) >> 8);
    ht4k_t* ht = (ht4k_t*)calloc(1, sizeof(ht4k_t));
    uint8_t* tmp = (uint8_t*)malloc(bmax + bmax / 2 + 64);
    size_t stream_off = 0;
    for (size_t off = 0; off < n; off += bmax) {
        size_t len = n - off < bmax ? n - off : bmax;
        sink_t s = {tmp, tmp + bmax + bmax / 2 + 64, 0};
        size_t comp = lzf_compress_internal(src + off, len, ht, stream_off, &s);
        if (!s.overflow && comp < len) { /* write_block: comp_len < src.len() -> Compressed */
            wr32(o, (uint32_t)comp); o += 4;
            memcpy(o, tmp, comp); o += comp;
        } else {
            wr32(o, (uint32_t)len | BLOCK_UNCOMPRESSED_BIT); o += 4;
            memcpy(o, src + off, len); o += len;
        }
        stream_off += len;
    }
    free(tmp);
    free(ht);
    wr32(o, 0); o += 4;
    wr32(o, or_xxh32(src, n, 0)); o += 4;
    *out_len = (size_t)(o - dst);
    return OR_OK;
}

/* ------------------------------------------------------ block decoder */
/* lz4_flex block/decompress_safe.rs decompress_internal semantics. out[0..hist) is
 * history the block may reference (linked blocks); the block writes from out+hist.
 * `limit` is the block's output limit (max block size); `cap` the caller's buffer end.
 * Overflowing `limit` is corruption; overflowing only `cap` is DST_TOO_SMALL. */
static int decode_block_impl(const uint8_t* in, size_t n, uint8_t* out, size_t hist,
                             size_t limit, size_t cap, size_t* produced) {
    size_t ip = 0, op = hist;
    size_t end = hist + limit;
    for (;;) {
        if (ip >= n) return OR_CORRUPT; /* expected a token */
        uint8_t t = in[ip++];
        size_t ll = t >> 4;
        if (ll == 15) {
            uint8_t b;
            do {
                if (ip >= n) return OR_CORRUPT;
                b = in[ip++];
                ll += b;
            } while (b == 255);
        }
        if (ll > n - ip) return OR_CORRUPT;
        if (ll > end - op) return OR_CORRUPT;
        if (op + ll > cap) return OR_DST_TOO_SMALL;
        memcpy(out + op, in + ip, ll);
        ip += ll;
        op += ll;
        if (ip >= n) break; /* last sequence: literals only */
        if (n - ip < 2) return OR_CORRUPT;
        size_t off = (size_t)in[ip] | ((size_t)in[ip + 1] << 8);
        ip += 2;
        size_t ml = (size_t)(t & 15) + MINMATCH;
        if ((t & 15) == 15) {
            uint8_t b;
            do {
                if (ip >= n) return OR_CORRUPT;
                b = in[ip++];
                ml += b;
            } while (b == 255);
        }
        if (off == 0 || off > op) return OR_CORRUPT;
        if (ml > end - op) return OR_CORRUPT;
        if (op + ml > cap) return OR_DST_TOO_SMALL;
        for (size_t k = 0; k < ml; k++) out[op + k] = out[op - off + k]; /* overlap-safe */
        op += ml;
    }
    *produced = op - hist;
    return OR_OK;
}

int or_decode_block(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len) {
    return decode_block_impl(src, n, dst, 0, cap, cap, out_len);
}

/* ------------------------------------------------------- frame reader */
typedef struct {
    uint8_t flg, bd;
    size_t bmax;
    size_t hdr_len;
    uint64_t content_size;
} frame_hdr_t;

/* FrameInfo::read_size + FrameInfo::read + the dict-id rejection of read_frame_info. */
static int parse_header(const uint8_t* p, size_t avail, frame_hdr_t* h) {
    if (avail < 4) return OR_CORRUPT; /* UnexpectedEof */
    uint32_t magic = rd32(p);
    if (magic == LZ4F_LEGACY_MAGIC) return OR_UNSUPPORTED;
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) return OR_UNSUPPORTED; /* skippable frame */
    if (magic != LZ4F_MAGIC) return OR_CORRUPT;                      /* WrongMagicNumber */
    if (avail < 7) return OR_CORRUPT;
    uint8_t flg = p[4], bd = p[5];
    size_t need = 7;
    if (flg & FLG_CONTENT_SIZE) need += 8;
    if (flg & FLG_DICT_ID) need += 4;
    if (avail < need) return OR_CORRUPT;
    if ((flg & FLG_VERSION_MASK) != FLG_VERSION_01) return OR_CORRUPT;
    if ((flg & FLG_RESERVED) || (bd & BD_RESERVED)) return OR_CORRUPT;
    size_t bmax = block_size_of_code((bd >> 4) & 7);
    if (!bmax) return OR_CORRUPT;
    uint8_t hc = (uint8_t)(or_xxh32(p + 4, need - 5, 0) >> 8);
    if (hc != p[need - 1]) return OR_CORRUPT; /* HeaderChecksumError */
    if (flg & FLG_DICT_ID) return OR_UNSUPPORTED;
    h->flg = flg;
    h->bd = bd;
    h->bmax = bmax;
    h->hdr_len = need;
    h->content_size = (flg & FLG_CONTENT_SIZE) ? ((uint64_t)rd32(p + 6) | ((uint64_t)rd32(p + 10) << 32)) : 0;
    return OR_OK;
}

/* One FrameDecoder::read_to_end: decode a frame at src[*pos], append at dst[*op]. */
static int decode_frame(const uint8_t* src, size_t n, size_t* pos, uint8_t* dst, size_t cap,
                        size_t* op, size_t* produced) {
    frame_hdr_t h;
    int rc = parse_header(src + *pos, n - *pos, &h);
    if (rc) return rc;
    size_t ip = *pos + h.hdr_len;
    size_t frame_out = *op;
    for (;;) {
        if (n - ip < 4) return OR_CORRUPT;
        uint32_t w = rd32(src + ip);
        ip += 4;
        if (w == 0) { /* EndMark */
            size_t got = *op - frame_out;
            if ((h.flg & FLG_CONTENT_SIZE) && got != h.content_size) return OR_CORRUPT;
            if (h.flg & FLG_CONTENT_CHECKSUM) {
                if (n - ip < 4) return OR_CORRUPT;
                uint32_t want = rd32(src + ip);
                ip += 4;
                if (or_xxh32(dst + frame_out, got, 0) != want) return OR_CHECKSUM;
            }
            *pos = ip;
            *produced = got;
            return OR_OK;
        }
        size_t len = w & 0x7FFFFFFFu;
        int stored = (w & BLOCK_UNCOMPRESSED_BIT) != 0;
        if (len > h.bmax) return OR_CORRUPT; /* BlockTooBig */
        if (n - ip < len) return OR_CORRUPT;
        if (h.flg & FLG_BLOCK_CHECKSUM) {
            if (n - ip - len < 4) return OR_CORRUPT;
            if (or_xxh32(src + ip, len, 0) != rd32(src + ip + len)) return OR_CHECKSUM;
        }
        if (stored) {
            if (cap - *op < len) return OR_DST_TOO_SMALL;
            memcpy(dst + *op, src + ip, len);
            *op += len;
        } else {
            /* Independent: history = this block only. Linked: the frame's earlier output. */
            size_t hist = (h.flg & FLG_INDEPENDENT) ? 0 : (*op - frame_out);
            size_t got = 0;
            rc = decode_block_impl(src + ip, len, dst + (*op - hist), hist, h.bmax, cap - (*op - hist), &got);
            if (rc) return rc;
            *op += got;
        }
        ip += len;
        if (h.flg & FLG_BLOCK_CHECKSUM) ip += 4;
    }
}

/* compression.rs:463-502 */
int or_decompress_data(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_len) {
    size_t pos = 0, op = 0;
    while (pos < n) {             /* :474-477 */
        size_t produced = 0;
        int rc = decode_frame(src, n, &pos, dst, cap, &op, &produced);
        if (rc) return rc;        /* :483-492 */
        if (produced == 0) break; /* :481 Ok(0) => break */
    }
    *out_len = op;
    return OR_OK;
}

size_t or_decompressed_bound(const uint8_t* src, size_t n) {
    size_t pos = 0, bound = 0;
    while (pos < n) {
        frame_hdr_t h;
        if (parse_header(src + pos, n - pos, &h)) return bound;
        size_t ip = pos + h.hdr_len;
        for (;;) {
            if (n - ip < 4) return bound;
            uint32_t w = rd32(src + ip);
            ip += 4;
            if (w == 0) {
                if (h.flg & FLG_CONTENT_CHECKSUM) ip += 4;
                break;
            }
            size_t len = w & 0x7FFFFFFFu;
            bound += (w & BLOCK_UNCOMPRESSED_BIT) ? len : h.bmax;
            ip += len + ((h.flg & FLG_BLOCK_CHECKSUM) ? 4 : 0);
            if (ip > n) return bound;
        }
        pos = ip;
    }
    return bound;
}

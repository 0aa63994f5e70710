// s3hc_plan.hpp — descriptors shared by the host planner and the CDNA4 kernels.
//
// The GPU engine works on three granularities:
//   frame   — one LZ4 frame (magic, FLG, BD, HC, blocks, EndMark, xxh32 content checksum)
//   block   — one LZ4 block inside a frame (<= 64 KiB, 256 KiB or 4 MiB, frame BD decides)
//   segment — kSeg input bytes of one block; the unit of parallel match finding on encode
#pragma once
#include <stdint.h>

namespace s3hc {

constexpr uint32_t kMagic = 0x184D2204u;         // compression.rs:50 LZ4F_MAGIC_NUMBER
constexpr uint32_t kStoredBit = 0x80000000u;     // compression.rs:47 BLOCK_UNCOMPRESSED_SIZE_BIT
constexpr uint32_t kStoreModeBlock = 4u << 20;   // compression.rs:42 STORE_MODE_MAX_BLOCK_SIZE
constexpr uint8_t kFlgIndependentChecksum = 0x64;  // version 01 | independent | content checksum

// ---- encode -------------------------------------------------------------
constexpr uint32_t kSeg = 4096;          // bytes of input per match-finding wave
// kernel-only tuning constants (diagnostic builds may override them; the host never reads them)
#ifndef S3HC_PREWARM
#define S3HC_PREWARM 4096
#endif
#ifndef S3HC_HASHLOG
#define S3HC_HASHLOG 11
#endif
constexpr uint32_t kPrewarm = S3HC_PREWARM;  // bytes before a segment inserted into its hash table
constexpr uint32_t kHashLog = S3HC_HASHLOG;  // per-wave hash table: 2^11 x u16 positions
constexpr uint32_t kMaxSeqPerSeg = kSeg / 4 + 1;
#ifndef S3HC_GROUP_SEGS
#define S3HC_GROUP_SEGS 8
#endif
constexpr uint32_t kGroupSegs = S3HC_GROUP_SEGS;  // segments (waves) per match-finding workgroup

enum : uint32_t {
    EB_STORE = 1,        // write this block stored (store-mode frame or caller decision)
    EB_FIRST = 2,        // first block of its frame: frame header precedes it
    EB_LAST = 4,         // last block of its frame: EndMark + content checksum follow it
    EB_EMPTY = 8,        // zero-length frame: header + EndMark + checksum only, no block
};

struct EncBlock {        // 40 bytes
    uint64_t src_off;    // input byte offset of this block
    uint32_t len;        // input bytes (<= block max of the frame)
    uint32_t seg0;       // first segment index
    uint32_t nseg;       // segments covering the block (>= 1)
    uint32_t frame;      // owning frame
    uint32_t flags;      // EB_*
    uint8_t  bd;         // frame BD byte (written in the header when EB_FIRST)
    uint8_t  hc;         // frame header checksum byte
    uint8_t  pad[6];
};

struct SegSummary {      // written by k_enc_parse, read by k_enc_sizes / k_enc_emit
    uint32_t nseq;       // sequences (matches) found in the segment
    uint32_t ll0;        // literal bytes of the first sequence that lie inside the segment
    uint32_t body;       // encoded bytes of all sequences minus the first token/literal-length run
    uint32_t trail;      // literal bytes after the last match (carried into the next segment)
};

struct SegPlace {        // written by k_enc_sizes
    uint32_t out_off;    // offset of this segment's first byte inside the block payload
    uint32_t carry;      // literal bytes carried in from earlier segments (nseq > 0 only)
};

// ---- decode -------------------------------------------------------------
enum : uint32_t {
    DB_STORED = 1,       // stored (uncompressed) block
    DB_LINKED = 2,       // linked-block frame: matches may reach into earlier blocks of the unit
};

struct DecBlock {        // 40 bytes
    uint64_t src_off;    // payload offset in the compressed stream
    uint64_t dst_off;    // output offset (first block of a unit); later blocks follow contiguously
    uint32_t csize;      // payload bytes
    uint32_t limit;      // frame max block size (more decoded bytes = corrupt frame)
    uint32_t cap;        // room in the caller's buffer at dst_off (more = DST_TOO_SMALL)
    uint32_t flags;      // DB_*
    uint32_t frame;      // owning frame
    uint32_t tok;        // 64 KiB fast path: first entry of this block's token-position slot in
                         // FastArgs::rec (slots sized by compressed bytes: (csize - 1) / 3 + 1
                         // entries, disjoint per block of a launch; see tok_slot_entries)
};

// Token-position slots of the fast path (s3hc_fast.hip): a block of c compressed bytes has at most
// (c - 1) / 3 + 1 tokens. Device plans give frame f the entries [ftok[f], ftok[f] + len_f / 3 + 2)
// and a block at byte ip of its frame the slot ftok[f] + ip / 3: blocks of a frame are >= 4 bytes
// apart, so their slots are disjoint (floor(a/3) + floor((c-1)/3) + 1 <= floor((a + c + 2)/3)).
inline uint64_t tok_frame_entries(uint64_t frame_len) { return frame_len / 3 + 2; }
inline uint64_t tok_slot_entries(uint32_t csize) { return csize ? (uint64_t)(csize - 1) / 3 + 1 : 0; }

struct DecUnit {         // a run of blocks decoded in order by one wave
    uint32_t first;
    uint32_t n;
};

// ---- large-block decode ---------------------------------
// Blocks whose frame allows more than 64 KiB (BD 0x50 / 0x70: what lz4_flex writes for the
// reference's ~1 MiB cache batches) are decoded by a whole workgroup each instead of one wave:
// the token chain is found by speculative segment walks over 8 Ki-position chunks of the
// compressed block (all chunks of all blocks in parallel), the sequence table comes from scans, and one
// 1024-thread workgroup per block then writes the output in 7.5 KiB steps (15 waves, 8 bytes per
// lane), resolving each step's match chains in LDS by pointer jumping against a 64 KiB ring of
// recent output, while its 16th wave hashes the flushed output (the frame's content xxh32 when
// the block is the whole frame). Launches of few such blocks decode every 7.5 KiB tile at once
// instead (spread execution, k_lbw_*).
#ifndef S3HC_LB_CHUNK  // (diagnostic builds try other sizes)
#define S3HC_LB_CHUNK 8192  // A/B (tools_lbchunk_ab.sh): 1 MiB frame 0.98 -> 0.90 ms, 16 and 256 frames equal; 4096 loses at 256
#endif
constexpr uint32_t kLbChunk = S3HC_LB_CHUNK;  // compressed positions per tokenizing workgroup
constexpr uint32_t kLbTokSlot = kLbChunk / 3 + 2;  // tokens of one chunk, at most (nodes >= 3 apart)
#ifndef S3HC_LB_TOKV2  // 1: chunk chains by speculative segment walks (round 6); 0: next token at every
#define S3HC_LB_TOKV2 1  // position + pointer doubling (rounds 1-5; diagnostic builds, A/B)
#endif
#ifndef S3HC_LB_WALKT
#define S3HC_LB_WALKT 256
#endif
constexpr uint32_t kLbWalkT = S3HC_LB_WALKT;  // segment walks (threads) per chunk (S3HC_LB_TOKV2)
#ifndef S3HC_LB_WALKLEAD
#define S3HC_LB_WALKLEAD 1
#endif
constexpr uint32_t kLbWalkLead = S3HC_LB_WALKLEAD;  // segments a walk starts before its own (unmarked)
constexpr uint32_t kLbFirstX = 64;        // chunk-relative positions whose chain exit is tabulated
constexpr uint32_t kLbEPerChunk = S3HC_LB_TOKV2 ? kLbFirstX : kLbChunk;        // E entries per chunk
constexpr uint32_t kLbJ0PerChunk = S3HC_LB_TOKV2 ? 2 * (kLbChunk / 32 + 3 * kLbWalkT) : kLbChunk;  // J0 (u16) per chunk
constexpr uint32_t kLbStep = 7680;        // output bytes per step of the executing workgroup
#ifndef S3HC_LB_XBAR  // 1: k_lb_run's decoding waves synchronise by an LDS counter and its hashing wave
#define S3HC_LB_XBAR 1  // runs free (round 6); 0: every wave at every s_barrier (rounds 2-5; diag A/B)
#endif
#ifndef S3HC_LB_OWNFUSE  // 1: k_lb_run runs the next step's owner scan inside the jumping rounds (two
#define S3HC_LB_OWNFUSE S3HC_LB_XBAR  // barriers fewer per step when there are >= 3 rounds)
#endif
constexpr uint32_t kLbMaxSteps = 547;     // steps of one block (ceil(4 MiB / kLbStep))
constexpr uint32_t kLbMinLimit = 65537;   // frame max block size above 64 KiB selects the path
constexpr uint32_t kLbFewBlocks = 256;    // batches with at most this many blocks: every compressed
                                          // independent block takes the path (latency: one wave per
                                          // 64 KiB block needs 0.85 ms)
constexpr uint32_t kLbwRounds = 4;        // spread execution: pointer-jumping launches (k_lbw_gather
                                          // walks whatever chains they leave)
constexpr uint32_t kLbwHops = 8;          // ... hops per byte and launch, at most
constexpr uint32_t kLbwCapMax = 1u << 30; // spread execution: pointer-array positions, at most
constexpr uint32_t kLbwMaxBlocks = 16;        // ... and so do launches of more large blocks than this:
                                              // the step loop's one workgroup per block lets the reader's
                                              // queues overlap batches (config-4 A/B, §4b)
#ifndef S3HC_LBW_MINLIMIT  // (diagnostic builds try other values)
#define S3HC_LBW_MINLIMIT 65536
#endif
constexpr uint32_t kLbwMinLimit = S3HC_LBW_MINLIMIT;  // spread: blocks of frames allowing more than this
constexpr uint32_t kLbwMaxOut = 96u << 20;     // launches whose large blocks may decode to more than
                                              // this run the step loop (k_lb_run): with a block per CU
                                              // it is as fast, and P stays small (measured, §4b)

struct LbBlock {         // 48 bytes; one per block taken by the large-block path
    uint64_t src_off;    // compressed payload
    uint64_t dst_off;    // output
    uint32_t C, limit, cap;
    uint32_t blk;        // DecBlock index (blk_out / blk_status)
    uint32_t unit;       // DecUnit index (unit_lb flag)
    uint32_t chunk0, nchunks;
    uint32_t pad;
};

struct LbCtl {           // device-side counters of one large-block launch
    uint32_t nlb, nchunks, ntiles, pad0;
    uint32_t rflag[kLbwRounds + 2];  // spread execution: [r] = tiles still pending before round r
};

// Device scratch of the large-block path (sized by the host: lb_cap blocks, chunk_cap chunks;
// blocks beyond a cap are decoded by the one-wave decoder instead).
struct LbArgs {
    uint32_t lb_cap, chunk_cap;
    uint32_t min_limit;    // frame max block size that selects the path (kLbMinLimit; 1 for few-block batches)
    uint32_t wcap;         // spread execution: positions of P (0: every block runs the step loop)
    uint32_t tile_cap;     // spread execution: tiles (kLbStep output bytes) of the spread blocks, at most
    uint32_t all_spread;   // the host's bounds show every taken block runs spread: no k_lb_run launch
    uint32_t big_csize;    // a block of a frame allowing <= min_limit takes the path anyway when its
                           // compressed size exceeds this (small launches: blocks the fused fast
                           // path k_dsmall cannot take; 0xFFFFFFFF = never)
    LbBlock* lbt;
    LbCtl* ctl;
    uint8_t* unit_lb;      // per unit: 1 = decoded by this path
    uint32_t* chunk_blk;   // chunk -> LB block
    uint32_t* nzg;         // per chunk, per 64-byte granule: first non-255 byte at or after it (chunk-local)
    uint32_t* E;           // per chunk x kLbEPerChunk: chain exit of a chunk-relative position (walks: the
                           // first kLbFirstX positions; doubling tables: every position)
    uint16_t* J0;          // per chunk x kLbJ0PerChunk: walks: the walk-1 marks and segment exits (u32);
                           // doubling tables: next token inside the chunk per position
    uint32_t* entry;       // per chunk: first chain position (chunk-relative) or ~0
    uint4* trec;           // per chunk, kLbTokSlot slots: its tokens in order (lit | last << 31, ll, ml, off)
    uint32_t* ntok;        // per chunk: sequences
    uint32_t* slsum;       // per chunk: output bytes (saturating)
    uint32_t* badrel;      // per chunk: malformed token ending the chain, or ~0
    uint64_t* tokbase;     // exclusive scans of ntok / slsum
    uint64_t* outbase;
    uint64_t* total;       // scan totals (2 x u64)
    uint4* seq4;           // per sequence: out, lit, ll, ml
    uint16_t* seqoff;      // per sequence: match offset
    uint32_t* lb_err;      // per LB block: min(rank << 3 | status) of failing sequences
    uint32_t* lb_size;     // per LB block: decoded bytes (0 unless OK)
    uint32_t* lb_stat;     // per LB block: status
    uint32_t* lb_tok0;     // per LB block: global index of its first sequence
    uint32_t* lb_ntok;
    uint32_t* rfirst;      // per LB block x kLbMaxSteps: sequence covering each step's first byte
    uint64_t* blk_hash;    // per DecBlock: 1 << 32 | xxh32 of its output (written by k_lb_run; cleared
                           // by k_lb_classify for every single-block unit)
    // spread execution (few blocks): every byte of a block gets a source pointer
    // at once, chains are resolved by global pointer jumping over all tiles of all spread blocks
    uint32_t* wbase;       // per LB block: first position in P, or ~0 (the block runs k_lb_run)
    uint32_t* wtile0;      // per LB block: first tile (exclusive scan of the spread blocks' tiles)
    uint32_t* P;           // per output byte of the spread blocks: ~0 final, 1 << 31 | root, or source
    uint8_t* tpend;        // per tile: some byte still has a plain pointer
    uint8_t* tinit;        // per tile: some byte was left pending by k_lbw_init (needs the gather)
};

// ---- 64 KiB-block decode fast path ------------------------
// k_dtok finds every token of a block (speculative segment walks over the LDS-staged block,
// chains merged by pointer doubling) and validates the block against lz4_flex's bounds; it
// hands the token positions to k_dexec, which executes 64 sequences at a time, one per lane.
// Blocks it does not take (stored, > kFastMaxC compressed bytes, multi-block units, anything
// malformed or out of bounds) go to the per-unit decoder, which also reports their exact status.
constexpr uint32_t kFastMaxC = 32768;  // compressed bytes of a block the fast path takes
// tokens of such a block: every sequence but the last has a token and a 2-byte offset, the last
// a token and >= 1 literal, so N <= (C - 1) / 3 + 1 (rounded up to whole 64-token windows)
constexpr uint32_t kFastMaxTok = ((kFastMaxC - 1) / 3 + 1 + 63) / 64 * 64;

struct FastUnit {        // 16 bytes, written by k_dtok for every unit it takes
    uint32_t ntok;       // sequences (the last one has no match)
    uint32_t U;          // decoded bytes
    uint32_t pad0, pad1;
};

// k_dtok's dynamic LDS for blocks of at most maxc compressed bytes: the staged block (16-byte
// alignment slack + zero read-ahead) and one bitmap bit per compressed position
constexpr uint32_t fast_stage_bytes(uint32_t maxc) { return (maxc + 64u + 15u) & ~15u; }
constexpr uint32_t fast_lds_bytes(uint32_t maxc) { return fast_stage_bytes(maxc) + 4u * ((maxc + 31u) / 32u + 1u); }

struct FastArgs {
    uint2* rec;          // per block, at DecBlock::tok: the block's sequence records in stream order,
                         // {lit | ll << 15, off | (ml - 4) << 16} (off = 0: the last, match-less one)
    FastUnit* fu;        // per unit
    uint8_t* unit_fast;  // per unit: 1 = decoded by the fast path
    uint32_t maxc;       // largest compressed block of the launch (<= kFastMaxC: sizes k_dtok's LDS);
                         // 0 = no block for the fast path
    uint64_t* bh;        // per DecBlock (nullable): 1 << 32 | content xxh32 of a single-block unit the
                         // fast path decoded, 0 for the single-block units it left (frame close
                         // takes the hash instead of reading the frame's output again)
};

}  // namespace s3hc

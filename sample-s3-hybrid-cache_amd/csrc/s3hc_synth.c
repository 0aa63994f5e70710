// s3hc_synth.c — synthetic corpora for the benchmark configs, not codec code.
//
// The benchmark's inputs must be resident in HBM before timing, and config 5 asks for 8 GiB of
// distinct log text per GPU; a Python generator is far too slow for that. This file fills a
// host buffer with S3-proxy access-log lines or JSON records, in 1 MiB pieces that are
// generated independently (each from its own seed, starting at a fresh line) on host threads,
// so the output depends only on (n, seed), never on the thread count. Nothing here repeats:
// every line draws its own fields.
//
// Built into libs3hc_synth.so (gcc, pthreads); used by synth.py. No GPU, no codec.
#include <math.h>
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <unistd.h>

#define PIECE (1u << 20)

typedef struct {
    uint64_t s;
} rng_t;

static inline uint64_t rnext(rng_t* r) {  // splitmix64
    uint64_t z = (r->s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static inline uint32_t rbelow(rng_t* r, uint32_t n) { return (uint32_t)(((rnext(r) >> 32) * (uint64_t)n) >> 32); }
static inline double runif(rng_t* r) { return (double)((rnext(r) >> 11) + 1) * 0x1.0p-53; }  // (0, 1]

// ---- Zipf(a) mod K residue tables (numpy's rng.zipf(a) % K, tail beyond kZipfTerms spread evenly)
#define kZipfTerms 2000000
typedef struct {
    double a;
    uint32_t K;
    double* cdf;
} zipf_t;
static double g_cdf_store[5 + 7 + 5000 + 10];
static zipf_t g_zb = {1.6, 5, g_cdf_store};
static zipf_t g_zp = {1.4, 7, g_cdf_store + 5};
static zipf_t g_zk = {1.3, 5000, g_cdf_store + 12};
static zipf_t g_zu = {1.5, 10, g_cdf_store + 5012};
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void zipf_init(zipf_t* z) {
    double tot = 0.0;
    for (uint32_t r = 0; r < z->K; ++r) z->cdf[r] = 0.0;
    for (uint32_t k = 1; k <= kZipfTerms; ++k) {
        double p = pow((double)k, -z->a);
        z->cdf[k % z->K] += p;
        tot += p;
    }
    const double tail = pow((double)kZipfTerms, 1.0 - z->a) / (z->a - 1.0);
    tot += tail;
    double acc = 0.0;
    for (uint32_t r = 0; r < z->K; ++r) {
        acc += (z->cdf[r] + tail / z->K) / tot;
        z->cdf[r] = acc;
    }
    z->cdf[z->K - 1] = 1.0;
}
static void tables_init(void) {
    zipf_init(&g_zb);
    zipf_init(&g_zp);
    zipf_init(&g_zk);
    zipf_init(&g_zu);
}
static inline uint32_t zipf_draw(const zipf_t* z, rng_t* r) {
    const double u = runif(r) * (1.0 - 1e-15);
    uint32_t lo = 0, hi = z->K - 1;
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (z->cdf[mid] > u) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

// ---- text helpers
static inline char* put(char* p, const char* s) {
    size_t n = strlen(s);
    memcpy(p, s, n);
    return p + n;
}
static inline char* put_u64(char* p, uint64_t v, int width) {
    char tmp[24];
    int n = 0;
    do {
        tmp[n++] = (char)('0' + v % 10);
        v /= 10;
    } while (v);
    while (n < width) tmp[n++] = '0';
    while (n) *p++ = tmp[--n];
    return p;
}
static inline char* put2(char* p, uint32_t v) {
    p[0] = (char)('0' + v / 10);
    p[1] = (char)('0' + v % 10);
    return p + 2;
}

static const char* const kLevels[20] = {"INFO", "INFO", "INFO", "INFO", "INFO", "INFO", "INFO", "INFO", "INFO", "INFO",
                                        "INFO", "INFO", "DEBUG", "DEBUG", "DEBUG", "DEBUG", "DEBUG", "WARN", "WARN",
                                        "ERROR"};
static const char* const kMethods[20] = {"GET", "GET", "GET", "GET", "GET", "GET", "GET", "GET", "GET", "GET",
                                         "GET", "GET", "GET", "GET", "HEAD", "HEAD", "HEAD", "PUT", "PUT", "DELETE"};
static const char* const kBuckets[5] = {"datalake-prod", "ml-training", "logs-archive", "media-assets", "backup-east"};
static const char* const kPrefix[7] = {"2024/01/", "2024/02/", "raw/", "curated/parquet/", "images/thumbs/",
                                       "models/ckpt/", "events/"};
static const char* const kExt[8] = {".parquet", ".json", ".csv", ".jpg", ".bin", ".log", ".gz", ".txt"};
static const char* const kStatus[33] = {"200", "200", "200", "200", "200", "200", "200", "200", "200", "200", "200",
                                        "200", "200", "200", "200", "200", "200", "200", "200", "200", "206", "206",
                                        "206", "206", "206", "206", "304", "304", "304", "404", "403", "500", "503"};
static const char* const kUsers[10] = {"alice", "bob", "carol", "dave", "erin", "frank", "grace", "heidi", "ivan", "judy"};
static const char* const kTags[10] = {"hot", "cold", "archive", "pii", "public", "ml", "etl", "raw", "gold", "silver"};
static const char kHex[] = "0123456789abcdef";

// One line into p (<= 256 bytes); returns the end.
static char* log_line(char* p, rng_t* r, uint64_t* t) {
    *t += rbelow(r, 3);
    const uint64_t T = *t;
    p = put(p, "2024-01-");
    p = put2(p, (uint32_t)(1 + (T / 86400) % 28));
    *p++ = 'T';
    p = put2(p, (uint32_t)((T / 3600) % 24));
    *p++ = ':';
    p = put2(p, (uint32_t)((T / 60) % 60));
    *p++ = ':';
    p = put2(p, (uint32_t)(T % 60));
    *p++ = 'Z';
    *p++ = ' ';
    p = put(p, kLevels[rbelow(r, 20)]);
    p = put(p, " [req-");
    const uint64_t rid = rnext(r) >> 1;
    for (int k = 15; k >= 0; --k) *p++ = kHex[(rid >> (4 * k)) & 15];
    p = put(p, "] ");
    p = put(p, kMethods[rbelow(r, 20)]);
    p = put(p, " /");
    p = put(p, kBuckets[zipf_draw(&g_zb, r)]);
    *p++ = '/';
    p = put(p, kPrefix[zipf_draw(&g_zp, r)]);
    p = put(p, "part-");
    p = put_u64(p, zipf_draw(&g_zk, r), 5);
    p = put(p, kExt[rbelow(r, 8)]);
    p = put(p, " status=");
    p = put(p, kStatus[rbelow(r, 33)]);
    p = put(p, " bytes=");
    p = put_u64(p, rbelow(r, 1u << 26), 0);
    p = put(p, " latency_ms=");
    p = put_u64(p, (uint64_t)(-12.0 * (log(runif(r)) + log(runif(r)))), 0);
    *p++ = '\n';
    return p;
}

static char* json_line(char* p, rng_t* r, uint64_t* id) {
    *id += 1;
    p = put(p, "{\"id\":");
    p = put_u64(p, *id, 0);
    p = put(p, ",\"user\":\"");
    p = put(p, kUsers[zipf_draw(&g_zu, r)]);
    p = put(p, "\",\"tags\":[");
    const uint32_t nt = rbelow(r, 4);
    for (uint32_t j = 0; j < nt; ++j) {
        if (j) *p++ = ',';
        *p++ = '"';
        p = put(p, kTags[rbelow(r, 10)]);
        *p++ = '"';
    }
    p = put(p, "],\"ts\":");
    p = put_u64(p, 1704067200u + rbelow(r, 1735689600u - 1704067200u), 0);
    p = put(p, ",\"score\":0.");
    p = put_u64(p, rbelow(r, 1000000), 6);
    p = put(p, "}\n");
    return p;
}

typedef struct {
    uint8_t* out;
    size_t n;
    uint64_t seed;
    int kind;  // 0 log text, 1 json
    size_t next;  // next piece (under mu)
    pthread_mutex_t mu;
} job_t;

static void fill_piece(const job_t* J, size_t c) {
    const size_t lo = c * (size_t)PIECE;
    const size_t hi = lo + PIECE < J->n ? lo + PIECE : J->n;
    rng_t r = {J->seed * 0x2545F4914F6CDD1Dull + (uint64_t)c * 0x9E3779B97F4A7C15ull + 0x5EEDull};
    (void)rnext(&r);
    uint64_t t = 1704067200ull + (uint64_t)c * 8192ull;  // timestamps keep rising across pieces
    uint64_t id = (uint64_t)c * 16384ull;                 // ids too (json)
    char line[512];
    size_t o = lo;
    while (o < hi) {
        char* e = J->kind == 0 ? log_line(line, &r, &t) : json_line(line, &r, &id);
        size_t k = (size_t)(e - line);
        if (k > hi - o) k = hi - o;
        memcpy(J->out + o, line, k);
        o += k;
    }
}

static void* worker(void* arg) {
    job_t* J = (job_t*)arg;
    const size_t np = (J->n + PIECE - 1) / PIECE;
    for (;;) {
        pthread_mutex_lock(&J->mu);
        const size_t c = J->next++;
        pthread_mutex_unlock(&J->mu);
        if (c >= np) return NULL;
        fill_piece(J, c);
    }
}

static int run(uint8_t* out, size_t n, uint64_t seed, int kind, int threads) {
    pthread_once(&g_once, tables_init);
    if (!out && n) return 1;
    job_t J = {out, n, seed, kind, 0, PTHREAD_MUTEX_INITIALIZER};
    const size_t np = (n + PIECE - 1) / PIECE;
    if (threads <= 0) {
        long c = sysconf(_SC_NPROCESSORS_ONLN);
        threads = c > 16 ? 16 : (c < 1 ? 1 : (int)c);
    }
    if ((size_t)threads > np) threads = np ? (int)np : 1;
    pthread_t th[64];
    if (threads > 64) threads = 64;
    int started = 0;
    for (int i = 1; i < threads; ++i)
        if (pthread_create(&th[started], NULL, worker, &J) == 0) ++started;
    worker(&J);
    for (int i = 0; i < started; ++i) pthread_join(th[i], NULL);
    return 0;
}

int s3hc_synth_log_text(uint8_t* out, size_t n, uint64_t seed, int threads) { return run(out, n, seed, 0, threads); }
int s3hc_synth_json(uint8_t* out, size_t n, uint64_t seed, int threads) { return run(out, n, seed, 1, threads); }

/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called from the
 * product library (transformer-lm_amd/).  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may use it, and only as the checker.
 *
 * A plain-C restatement of the reference byte-level BPE path of gashon/transformer-lm:
 *   read      reference models/tokenizer/train.py:22  open(path,"r",encoding="utf-8").read()
 *   pretoken  reference models/tokenizer/train.py:143-146 (GPT-2 pattern, `regex` module)
 *   count     reference models/tokenizer/train.py:16-28   extract_subword_frequencies
 *   split     reference models/tokenizer/train.py:31-32   encode_subwords
 *   pairs     reference models/tokenizer/train.py:35-49   calculate_byte_pair_frequencies
 *   loop      reference models/tokenizer/train.py:183-228 (+ helpers 52-139)
 *   vocab     reference models/tokenizer/vocab.py:2-34
 *   encode    reference models/tokenizer/tokenizer.py:12-38, 63-138
 *
 * Semantics are the reference's exactly (pinned by tests/golden, generated from the
 * reference itself); the data structures differ for speed: the per-round
 * max(pairs, key=(count, pair)) of train.py:187-189 is a lazy max-heap ordered by
 * (count, bytes(a), bytes(b)), which returns the same pair because every present key
 * keeps an entry >= its current count (see the round loop in oracle_train_text).
 */
#include "bpe_oracle.h"

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "uclass_ranges.h"

/* ------------------------------------------------------------------ small utilities */
#define OR_GROW(ptr, cap, need)                                                   \
    do {                                                                          \
        if ((need) > (cap)) {                                                     \
            size_t nc_ = (cap) ? (cap) : 16;                                      \
            while (nc_ < (need)) nc_ *= 2;                                        \
            void* np_ = realloc((ptr), nc_ * sizeof(*(ptr)));                     \
            if (!np_) { fprintf(stderr, "oracle: out of memory\n"); abort(); }    \
            (ptr) = np_;                                                          \
            (cap) = nc_;                                                          \
        }                                                                         \
    } while (0)

static uint64_t hash_bytes(const uint8_t* p, size_t n) {
    uint64_t h = 0xcbf29ce484222325ULL ^ (n * 0x9E3779B97F4A7C15ULL);
    for (size_t i = 0; i < n; i++) { h ^= p[i]; h *= 0x100000001b3ULL; }
    h ^= h >> 29; h *= 0xBF58476D1CE4E5B9ULL; h ^= h >> 32;
    return h;
}
static uint64_t mix64(uint64_t z) {
    z ^= z >> 30; z *= 0xBF58476D1CE4E5B9ULL;
    z ^= z >> 27; z *= 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

typedef struct { uint8_t* p; size_t n, cap; } bbuf;   /* growable byte buffer */
static void bb_put(bbuf* b, const void* src, size_t n) {
    OR_GROW(b->p, b->cap, b->n + n);
    memcpy(b->p + b->n, src, n);
    b->n += n;
}
static void bb_u32(bbuf* b, uint32_t v) { bb_put(b, &v, 4); }
static void bb_u64(bbuf* b, uint64_t v) { bb_put(b, &v, 8); }

/* ------------------------------------------------------------ byte-string interning */
/* id -> bytes (arena offsets), bytes -> id (open addressing).  Used both for word
 * counting and for token identity: the reference identifies tokens by their bytes
 * (vocab.py:29, train.py:190, tokenizer.py:98-101). */
typedef struct {
    bbuf arena;
    size_t* off; uint32_t* len; int64_t* val; size_t n, cap_ids;
    int64_t* slots; size_t nslots;  /* slot -> id or -1 */
} strtab;

static void st_init(strtab* t, size_t nslots_pow2) {
    memset(t, 0, sizeof(*t));
    t->nslots = nslots_pow2;
    t->slots = malloc(t->nslots * sizeof(int64_t));
    for (size_t i = 0; i < t->nslots; i++) t->slots[i] = -1;
}
static void st_free(strtab* t) {
    free(t->arena.p); free(t->off); free(t->len); free(t->val); free(t->slots);
    memset(t, 0, sizeof(*t));
}
static const uint8_t* st_bytes(const strtab* t, size_t id) { return t->arena.p + t->off[id]; }
static void st_rehash(strtab* t) {
    size_t ns = t->nslots * 2;
    int64_t* s = malloc(ns * sizeof(int64_t));
    for (size_t i = 0; i < ns; i++) s[i] = -1;
    for (size_t id = 0; id < t->n; id++) {
        size_t h = hash_bytes(st_bytes(t, id), t->len[id]) & (ns - 1);
        while (s[h] >= 0) h = (h + 1) & (ns - 1);
        s[h] = (int64_t)id;
    }
    free(t->slots); t->slots = s; t->nslots = ns;
}
/* returns id; *created = 1 if new */
static size_t st_intern(strtab* t, const uint8_t* p, size_t n, int* created) {
    if ((t->n + 1) * 2 > t->nslots) st_rehash(t);
    size_t h = hash_bytes(p, n) & (t->nslots - 1);
    while (t->slots[h] >= 0) {
        size_t id = (size_t)t->slots[h];
        if (t->len[id] == n && memcmp(st_bytes(t, id), p, n) == 0) {
            if (created) *created = 0;
            return id;
        }
        h = (h + 1) & (t->nslots - 1);
    }
    OR_GROW(t->off, t->cap_ids, t->n + 1);
    t->len = realloc(t->len, t->cap_ids * sizeof(uint32_t));
    t->val = realloc(t->val, t->cap_ids * sizeof(int64_t));
    size_t id = t->n++;
    t->off[id] = t->arena.n;
    t->len[id] = (uint32_t)n;
    t->val[id] = 0;
    bb_put(&t->arena, p, n);
    t->slots[h] = (int64_t)id;
    if (created) *created = 1;
    return id;
}
static int64_t st_find(const strtab* t, const uint8_t* p, size_t n) {
    size_t h = hash_bytes(p, n) & (t->nslots - 1);
    while (t->slots[h] >= 0) {
        size_t id = (size_t)t->slots[h];
        if (t->len[id] == n && memcmp(st_bytes(t, id), p, n) == 0) return (int64_t)id;
        h = (h + 1) & (t->nslots - 1);
    }
    return -1;
}

/* --------------------------------------------------------------- text decoding */
/* Strict UTF-8 as CPython's "utf-8" codec (no surrogates, no overlongs, <= U+10FFFF),
 * then universal-newline translation \r\n -> \n, lone \r -> \n (text-mode read,
 * reference train.py:22).  Returns OR_E_UTF8 with *err_pos = first bad byte. */
static size_t utf8_seq_len(const uint8_t* s, size_t n, size_t i) {
    uint8_t b0 = s[i];
    if (b0 < 0x80) return 1;
    size_t need; uint8_t lo = 0x80, hi = 0xBF;
    if (b0 >= 0xC2 && b0 <= 0xDF) need = 2;
    else if (b0 == 0xE0) { need = 3; lo = 0xA0; }
    else if (b0 >= 0xE1 && b0 <= 0xEC) need = 3;
    else if (b0 == 0xED) { need = 3; hi = 0x9F; }
    else if (b0 >= 0xEE && b0 <= 0xEF) need = 3;
    else if (b0 == 0xF0) { need = 4; lo = 0x90; }
    else if (b0 >= 0xF1 && b0 <= 0xF3) need = 4;
    else if (b0 == 0xF4) { need = 4; hi = 0x8F; }
    else return 0;
    if (i + need > n) return 0;
    if (s[i + 1] < lo || s[i + 1] > hi) return 0;
    for (size_t k = 2; k < need; k++)
        if ((s[i + k] & 0xC0) != 0x80) return 0;
    return need;
}

int oracle_decode_text(const uint8_t* raw, size_t n, uint8_t** out, size_t* out_n,
                       size_t* err_pos) {
    for (size_t i = 0; i < n;) {
        size_t l = utf8_seq_len(raw, n, i);
        if (!l) { if (err_pos) *err_pos = i; return OR_E_UTF8; }
        i += l;
    }
    uint8_t* o = malloc(n ? n : 1);
    size_t j = 0;
    for (size_t i = 0; i < n; i++) {
        if (raw[i] == '\r') {
            o[j++] = '\n';
            if (i + 1 < n && raw[i + 1] == '\n') i++;
        } else {
            o[j++] = raw[i];
        }
    }
    *out = o; *out_n = j;
    return OR_OK;
}

/* --------------------------------------------------------- character classes */
enum { C_OTHER = 0, C_LETTER = 1, C_NUMBER = 2, C_SPACE = 3 };

static int in_ranges(const oracle_range* r, size_t n, uint32_t cp) {
    size_t lo = 0, hi = n;
    while (lo < hi) {
        size_t mid = (lo + hi) / 2;
        if (cp < r[mid].lo) hi = mid;
        else if (cp > r[mid].hi) lo = mid + 1;
        else return 1;
    }
    return 0;
}
static int cp_class(uint32_t cp) {
    if (in_ranges(ORACLE_S, sizeof ORACLE_S / sizeof ORACLE_S[0], cp)) return C_SPACE;
    if (in_ranges(ORACLE_L, sizeof ORACLE_L / sizeof ORACLE_L[0], cp)) return C_LETTER;
    if (in_ranges(ORACLE_N, sizeof ORACLE_N / sizeof ORACLE_N[0], cp)) return C_NUMBER;
    return C_OTHER;
}
/* decode the (already validated) code point at byte i; returns its byte length */
static size_t cp_at(const uint8_t* s, size_t i, uint32_t* cp) {
    uint8_t b = s[i];
    if (b < 0x80) { *cp = b; return 1; }
    if (b < 0xE0) { *cp = ((uint32_t)(b & 0x1F) << 6) | (s[i + 1] & 0x3F); return 2; }
    if (b < 0xF0) {
        *cp = ((uint32_t)(b & 0x0F) << 12) | ((uint32_t)(s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F);
        return 3;
    }
    *cp = ((uint32_t)(b & 0x07) << 18) | ((uint32_t)(s[i + 1] & 0x3F) << 12) |
          ((uint32_t)(s[i + 2] & 0x3F) << 6) | (s[i + 3] & 0x3F);
    return 4;
}

/* ------------------------------------------------------------ GPT-2 pretokenizer */
/* One leftmost-first match of
 *   '(?:[sdmt]|ll|ve|re)| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+
 * starting at byte p of the (sub)string s[0..n).  Returns the end offset. */
static size_t match_end(const uint8_t* s, size_t n, size_t p) {
    uint32_t c0;
    size_t l0 = cp_at(s, p, &c0);
    if (c0 == '\'' && p + 1 < n) {                         /* alternative 1 */
        uint8_t c1 = s[p + 1];
        if (c1 == 's' || c1 == 'd' || c1 == 'm' || c1 == 't') return p + 2;
        if (p + 2 < n) {
            uint8_t c2 = s[p + 2];
            if ((c1 == 'l' && c2 == 'l') || (c1 == 'v' && c2 == 'e') || (c1 == 'r' && c2 == 'e'))
                return p + 3;
        }
    }
    /* alternatives 2-4: an optional U+0020 then a run of one class */
    size_t q = p;
    int k;
    if (c0 == ' ' && p + 1 < n) {
        uint32_t c1;
        cp_at(s, p + 1, &c1);
        k = cp_class(c1);
        if (k != C_SPACE) q = p + 1;
    } else {
        k = cp_class(c0);
    }
    if (k != C_SPACE && !(q == p && c0 == ' ')) {
        size_t e = q;
        while (e < n) {
            uint32_t c;
            size_t l = cp_at(s, e, &c);
            if (cp_class(c) != k) break;
            e += l;
        }
        return e;
    }
    /* alternatives 5 and 6: a whitespace run; give back its last char if \S follows */
    size_t e = p + l0, last = p, cnt = 1;
    while (e < n) {
        uint32_t c;
        size_t l = cp_at(s, e, &c);
        if (cp_class(c) != C_SPACE) break;
        last = e; e += l; cnt++;
    }
    if (e == n) return e;
    return cnt >= 2 ? last : e;
}

typedef void (*span_fn)(void* ctx, size_t start, size_t len);
static void pretokenize(const uint8_t* s, size_t n, span_fn fn, void* ctx) {
    for (size_t p = 0; p < n;) {
        size_t e = match_end(s, n, p);
        fn(ctx, p, e - p);
        p = e;
    }
}

/* ------------------------------------------------------------ specials list */
typedef struct { const uint8_t** p; size_t* n; size_t count; } speclist;

static int parse_specials(const uint8_t* blob, size_t blob_n, speclist* sl) {
    memset(sl, 0, sizeof(*sl));
    if (!blob || blob_n < 4) return OR_OK;
    uint32_t cnt; memcpy(&cnt, blob, 4);
    sl->p = malloc((cnt + 1) * sizeof(*sl->p));
    sl->n = malloc((cnt + 1) * sizeof(*sl->n));
    size_t off = 4;
    for (uint32_t i = 0; i < cnt; i++) {
        if (off + 4 > blob_n) return OR_E_ARG;
        uint32_t l; memcpy(&l, blob + off, 4); off += 4;
        if (off + l > blob_n) return OR_E_ARG;
        sl->p[i] = blob + off; sl->n[i] = l; off += l;
    }
    sl->count = cnt;
    return OR_OK;
}
static int is_special(const speclist* sl, const uint8_t* p, size_t n) {
    for (size_t i = 0; i < sl->count; i++)
        if (sl->n[i] == n && memcmp(sl->p[i], p, n) == 0) return 1;
    return 0;
}

/* ------------------------------------------------------------ word counting */
typedef struct { const uint8_t* text; strtab* words; const speclist* sp; } count_ctx;
static void count_span(void* vctx, size_t start, size_t len) {
    count_ctx* c = vctx;
    if (is_special(c->sp, c->text + start, len)) return;      /* train.py:25 */
    size_t id = st_intern(c->words, c->text + start, len, NULL);
    c->words->val[id] += 1;                                    /* train.py:26 */
}

static void count_words(const uint8_t* text, size_t n, const speclist* sp, strtab* words) {
    st_init(words, 1 << 12);
    count_ctx c = {text, words, sp};
    pretokenize(text, n, count_span, &c);
}

/* --------------------------------------------------------------- pair table */
typedef struct { uint64_t key; int64_t count; uint8_t used, present; } pslot;
typedef struct { pslot* s; size_t cap, used; } ptab;

static void pt_init(ptab* t) { t->cap = 1 << 14; t->used = 0; t->s = calloc(t->cap, sizeof(pslot)); }
static pslot* pt_get(ptab* t, uint64_t key, int create);
static void pt_grow(ptab* t) {
    ptab nt = {calloc(t->cap * 2, sizeof(pslot)), t->cap * 2, 0};
    for (size_t i = 0; i < t->cap; i++)
        if (t->s[i].used) { pslot* d = pt_get(&nt, t->s[i].key, 1); *d = t->s[i]; }
    free(t->s); *t = nt;
}
static pslot* pt_get(ptab* t, uint64_t key, int create) {
    if (create && (t->used + 1) * 2 > t->cap) pt_grow(t);
    size_t h = mix64(key) & (t->cap - 1);
    while (t->s[h].used) {
        if (t->s[h].key == key) return &t->s[h];
        h = (h + 1) & (t->cap - 1);
    }
    if (!create) return NULL;
    t->s[h].used = 1; t->s[h].key = key; t->s[h].count = 0; t->s[h].present = 0;
    t->used++;
    return &t->s[h];
}
#define PKEY(a, b) (((uint64_t)(uint32_t)(a) << 32) | (uint32_t)(b))

/* ------------------------------------------------------------ lazy max-heap */
typedef struct { int64_t count; uint32_t a, b; } hent;
typedef struct { hent* h; size_t n, cap; const strtab* tok; } heap;

static int tok_cmp(const strtab* t, uint32_t x, uint32_t y) {   /* Python bytes ordering */
    if (x == y) return 0;
    size_t lx = t->len[x], ly = t->len[y];
    int c = memcmp(st_bytes(t, x), st_bytes(t, y), lx < ly ? lx : ly);
    if (c) return c;
    return lx < ly ? -1 : (lx > ly ? 1 : 0);
}
/* >0 if e1 ranks above e2 under key (count, (bytes a, bytes b)) of train.py:188 */
static int hent_cmp(const strtab* t, const hent* e1, const hent* e2) {
    if (e1->count != e2->count) return e1->count > e2->count ? 1 : -1;
    int c = tok_cmp(t, e1->a, e2->a);
    if (c) return c;
    return tok_cmp(t, e1->b, e2->b);
}
static void heap_push(heap* hp, int64_t count, uint32_t a, uint32_t b) {
    OR_GROW(hp->h, hp->cap, hp->n + 1);
    size_t i = hp->n++;
    hent e = {count, a, b};
    while (i > 0) {
        size_t par = (i - 1) / 2;
        if (hent_cmp(hp->tok, &hp->h[par], &e) >= 0) break;
        hp->h[i] = hp->h[par]; i = par;
    }
    hp->h[i] = e;
}
static hent heap_pop(heap* hp) {
    hent top = hp->h[0];
    hent e = hp->h[--hp->n];
    size_t i = 0;
    for (;;) {
        size_t l = 2 * i + 1, r = l + 1, m = i;
        const hent* best = &e;
        if (l < hp->n && hent_cmp(hp->tok, &hp->h[l], best) > 0) { m = l; best = &hp->h[l]; }
        if (r < hp->n && hent_cmp(hp->tok, &hp->h[r], best) > 0) { m = r; }
        if (m == i) break;
        hp->h[i] = hp->h[m]; i = m;
    }
    if (hp->n) hp->h[i] = e;
    return top;
}

/* ------------------------------------------------------------ trainer state */
typedef struct { uint32_t* t; uint32_t len, cap; int64_t count; uint64_t stamp; } oword;
typedef struct { uint32_t* w; uint32_t n, cap; } wlist;

typedef struct {
    strtab tok;          /* token id <-> bytes; ids 0..255 = single bytes */
    oword* words; size_t nwords;
    ptab pairs;
    heap hp;
} trainer;

/* The inverted index is keyed by pair key in its own table so that pair-table growth
 * does not invalidate it. */
typedef struct { uint64_t key; wlist l; uint8_t used; } islot;
typedef struct { islot* s; size_t cap, used; } itab;
static islot* it_get(itab* t, uint64_t key, int create);
static void it_grow(itab* t) {
    itab nt = {calloc(t->cap * 2, sizeof(islot)), t->cap * 2, 0};
    for (size_t i = 0; i < t->cap; i++)
        if (t->s[i].used) { islot* d = it_get(&nt, t->s[i].key, 1); *d = t->s[i]; }
    free(t->s); *t = nt;
}
static islot* it_get(itab* t, uint64_t key, int create) {
    if (create && (t->used + 1) * 2 > t->cap) it_grow(t);
    size_t h = mix64(key ^ 0x5555) & (t->cap - 1);
    while (t->s[h].used) {
        if (t->s[h].key == key) return &t->s[h];
        h = (h + 1) & (t->cap - 1);
    }
    if (!create) return NULL;
    memset(&t->s[h], 0, sizeof(islot));
    t->s[h].used = 1; t->s[h].key = key;
    t->used++;
    return &t->s[h];
}
static void it_add(itab* t, uint64_t key, uint32_t w) {
    islot* s = it_get(t, key, 1);
    OR_GROW(s->l.w, s->l.cap, s->l.n + 1);
    s->l.w[s->l.n++] = w;
}

/* frequencies[p] += c   (defaultdict semantics: a missing key is created at 0) */
static void pair_add(ptab* pt, heap* hp, uint32_t a, uint32_t b, int64_t c) {
    pslot* s = pt_get(pt, PKEY(a, b), 1);
    int created = !s->present;
    if (created) { s->present = 1; s->count = 0; }
    s->count += c;
    /* an increment (or a key just created) needs a heap entry at its new count; a
     * decrement leaves an older entry >= the current count, which the round loop re-pushes when popped */
    if (c > 0 || created) heap_push(hp, s->count, a, b);
}

/* ------------------------------------------------------------ Vocab (vocab.py) */
typedef struct { strtab set; } ovocab;   /* insertion order == id order */
static void vocab_add(ovocab* v, const uint8_t* p, size_t n) { st_intern(&v->set, p, n, NULL); }

/* ------------------------------------------------------------ train */
/* The merge loop of train.py:155-231 over a word -> count table (`words` is consumed). */
static int train_words(strtab* words_in, const speclist* spp, int vocab_size, oracle_blob* out) {
    const speclist sp = *spp;
    strtab words = *words_in;
    memset(words_in, 0, sizeof(*words_in));

    /* Vocab(special_tokens): specials in order, then the 256 bytes, deduplicated (vocab.py:2-12) */
    ovocab V; st_init(&V.set, 1 << 10);
    for (size_t i = 0; i < sp.count; i++) vocab_add(&V, sp.p[i], sp.n[i]);
    for (int b = 0; b < 256; b++) { uint8_t x = (uint8_t)b; vocab_add(&V, &x, 1); }
    long rounds = (long)vocab_size - (long)V.set.n;          /* train.py:183 */

    trainer T; memset(&T, 0, sizeof(T));
    st_init(&T.tok, 1 << 10);
    for (int b = 0; b < 256; b++) { uint8_t x = (uint8_t)b; st_intern(&T.tok, &x, 1, NULL); }
    T.hp.tok = &T.tok;
    pt_init(&T.pairs);
    itab idx = {calloc(1 << 14, sizeof(islot)), 1 << 14, 0};

    /* encode_subwords + calculate_byte_pair_frequencies (train.py:31-49) */
    T.nwords = words.n;
    T.words = calloc(words.n ? words.n : 1, sizeof(oword));
    for (size_t w = 0; w < words.n; w++) {
        oword* ow = &T.words[w];
        ow->len = ow->cap = words.len[w];
        ow->t = malloc((ow->len ? ow->len : 1) * sizeof(uint32_t));
        const uint8_t* wb = st_bytes(&words, w);
        for (uint32_t i = 0; i < ow->len; i++) ow->t[i] = wb[i];
        ow->count = words.val[w];
        for (uint32_t i = 0; i + 1 < ow->len; i++) {
            pslot* s = pt_get(&T.pairs, PKEY(ow->t[i], ow->t[i + 1]), 1);
            s->present = 1;
            s->count += ow->count;
            it_add(&idx, PKEY(ow->t[i], ow->t[i + 1]), (uint32_t)w);
        }
    }
    for (size_t i = 0; i < T.pairs.cap; i++)
        if (T.pairs.s[i].used)
            heap_push(&T.hp, T.pairs.s[i].count, (uint32_t)(T.pairs.s[i].key >> 32),
                      (uint32_t)T.pairs.s[i].key);

    bbuf mbuf = {0}; uint32_t nmerges = 0;
    uint64_t stamp = 0;
    uint8_t* cat = NULL; size_t catcap = 0;
    for (long r = 0; r < rounds; r++) {
        /* `if len(byte_pair_frequencies) == 0: break` (train.py:184-185) plus the max of
         * train.py:187-189 via the lazy heap */
        hent best; int found = 0;
        while (T.hp.n) {
            hent e = heap_pop(&T.hp);
            pslot* s = pt_get(&T.pairs, PKEY(e.a, e.b), 0);
            if (!s || !s->present) continue;
            if (s->count == e.count) { best = e; found = 1; break; }
            if (s->count < e.count) heap_push(&T.hp, s->count, e.a, e.b);
        }
        if (!found) break;
        uint32_t a = best.a, b = best.b;
        size_t la = T.tok.len[a], lb = T.tok.len[b];
        OR_GROW(cat, catcap, la + lb);
        memcpy(cat, st_bytes(&T.tok, a), la);
        memcpy(cat + la, st_bytes(&T.tok, b), lb);
        uint32_t nw = (uint32_t)st_intern(&T.tok, cat, la + lb, NULL);  /* new_byte (190) */
        vocab_add(&V, cat, la + lb);                                      /* add_token (191) */
        /* record merge (a_bytes, b_bytes) */
        bb_u32(&mbuf, (uint32_t)la); bb_put(&mbuf, st_bytes(&T.tok, a), la);
        bb_u32(&mbuf, (uint32_t)lb); bb_put(&mbuf, st_bytes(&T.tok, b), lb);
        nmerges++;

        islot* is = it_get(&idx, PKEY(a, b), 0);
        stamp++;
        size_t nlist = is ? is->l.n : 0;
        for (size_t li = 0; li < nlist; li++) {
            uint32_t wi = is->l.w[li];
            oword* w = &T.words[wi];
            if (w->stamp == stamp) continue;   /* token_indices[pair] is a dict keyed by word */
            w->stamp = stamp;
            int64_t c = w->count;
            for (uint32_t i = 0; i + 1 < w->len; i++) {           /* train.py:196-224 */
                if (w->t[i] == a && w->t[i + 1] == b) {
                    /* update_frequencies_after_merge (train.py:52-78), on the current word */
                    if (i > 0) {
                        pair_add(&T.pairs, &T.hp, w->t[i - 1], w->t[i], -c);
                        pair_add(&T.pairs, &T.hp, w->t[i - 1], nw, c);
                    }
                    if (i + 2 < w->len) {
                        pair_add(&T.pairs, &T.hp, w->t[i + 1], w->t[i + 2], -c);
                        pair_add(&T.pairs, &T.hp, nw, w->t[i + 2], c);
                    }
                    /* update_token_indices (81-104) never deletes */
                    /* merge_subwords (132-139) */
                    w->t[i] = nw;
                    memmove(&w->t[i + 1], &w->t[i + 2], (w->len - i - 2) * sizeof(uint32_t));
                    w->len--;
                    /* create_new_token_indices (107-129) */
                    if (i > 0) it_add(&idx, PKEY(w->t[i - 1], w->t[i]), wi);
                    if (i + 1 < w->len) it_add(&idx, PKEY(w->t[i], w->t[i + 1]), wi);
                    is = it_get(&idx, PKEY(a, b), 0);   /* it_add may have rehashed */
                }
            }
        }
        /* byte_pair_frequencies.pop(best_pair); token_indices.pop(best_pair) (226-227) */
        pslot* bs = pt_get(&T.pairs, PKEY(a, b), 0);
        bs->present = 0; bs->count = 0;
        is = it_get(&idx, PKEY(a, b), 0);
        if (is) is->l.n = 0;
    }

    /* output blob: u32 nmerges, merges..., u32 nvocab, vocab... */
    bbuf ob = {0};
    bb_u32(&ob, nmerges);
    bb_put(&ob, mbuf.p, mbuf.n);
    bb_u32(&ob, (uint32_t)V.set.n);
    for (size_t i = 0; i < V.set.n; i++) {
        bb_u32(&ob, V.set.len[i]);
        bb_put(&ob, st_bytes(&V.set, i), V.set.len[i]);
    }
    out->data = ob.p; out->n = ob.n;

    free(mbuf.p); free(cat);
    for (size_t w = 0; w < T.nwords; w++) free(T.words[w].t);
    free(T.words);
    for (size_t i = 0; i < idx.cap; i++) if (idx.s[i].used) free(idx.s[i].l.w);
    free(idx.s);
    free(T.pairs.s); free(T.hp.h);
    st_free(&T.tok); st_free(&words); st_free(&V.set);
    return OR_OK;
}

int oracle_train_text(const uint8_t* text, size_t n, int vocab_size,
                      const uint8_t* specials_blob, size_t specials_n, oracle_blob* out) {
    speclist sp;
    int rc = parse_specials(specials_blob, specials_n, &sp);
    if (rc) return rc;
    strtab words;
    count_words(text, n, &sp, &words);                        /* train.py:155 */
    rc = train_words(&words, &sp, vocab_size, out);
    free(sp.p); free(sp.n);
    return rc;
}

/* ------------------------------------------------------------ chunked counting */
/* extract_subword_frequencies (train.py:16-28) over a corpus fed in pieces.  Each piece must
 * end at a safe split point (a U+0020 between two ASCII non-space bytes, as
 * bpe_safe_split and the synthetic generator's 4 KiB block boundaries are): cutting there
 * changes neither the pre-token multiset nor the \r\n translation, so the sum of the
 * pieces' counts equals the whole text's. */
struct oracle_counter {
    speclist sp;
    uint8_t* sp_blob;
    strtab words;
};

oracle_counter* oracle_counter_new(const uint8_t* specials_blob, size_t specials_n) {
    oracle_counter* c = calloc(1, sizeof(*c));
    c->sp_blob = malloc(specials_n ? specials_n : 1);
    if (specials_n) memcpy(c->sp_blob, specials_blob, specials_n);
    if (parse_specials(c->sp_blob, specials_n, &c->sp)) { free(c->sp_blob); free(c); return NULL; }
    st_init(&c->words, 1 << 12);
    return c;
}

int oracle_counter_feed(oracle_counter* c, const uint8_t* raw, size_t n, size_t* err_pos) {
    uint8_t* text; size_t tn;
    int rc = oracle_decode_text(raw, n, &text, &tn, err_pos);
    if (rc) return rc;
    count_ctx cc = {text, &c->words, &c->sp};
    pretokenize(text, tn, count_span, &cc);
    free(text);
    return OR_OK;
}

int oracle_counter_absorb(oracle_counter* dst, const oracle_counter* src) {
    for (size_t i = 0; i < src->words.n; i++) {
        size_t id = st_intern(&dst->words, st_bytes(&src->words, i), src->words.len[i], NULL);
        dst->words.val[id] += src->words.val[i];
    }
    return OR_OK;
}

int oracle_counter_words(const oracle_counter* c, oracle_blob* out) {
    bbuf ob = {0};
    bb_u32(&ob, (uint32_t)c->words.n);
    for (size_t i = 0; i < c->words.n; i++) {
        bb_u32(&ob, c->words.len[i]);
        bb_put(&ob, st_bytes(&c->words, i), c->words.len[i]);
        bb_u64(&ob, (uint64_t)c->words.val[i]);
    }
    out->data = ob.p; out->n = ob.n;
    return OR_OK;
}

int oracle_counter_train(oracle_counter* c, int vocab_size, oracle_blob* out) {
    int rc = train_words(&c->words, &c->sp, vocab_size, out);
    st_init(&c->words, 1 << 12);
    return rc;
}

void oracle_counter_free(oracle_counter* c) {
    if (!c) return;
    st_free(&c->words);
    free(c->sp.p); free(c->sp.n); free(c->sp_blob);
    free(c);
}

int oracle_train_raw(const uint8_t* raw, size_t n, int vocab_size, const uint8_t* specials_blob,
                     size_t specials_n, oracle_blob* out, size_t* err_pos) {
    uint8_t* text; size_t tn;
    int rc = oracle_decode_text(raw, n, &text, &tn, err_pos);
    if (rc) return rc;
    rc = oracle_train_text(text, tn, vocab_size, specials_blob, specials_n, out);
    free(text);
    return rc;
}

/* ------------------------------------------------------------ word counts / spans */
int oracle_word_counts(const uint8_t* text, size_t n, const uint8_t* specials_blob,
                       size_t specials_n, oracle_blob* out) {
    speclist sp;
    int rc = parse_specials(specials_blob, specials_n, &sp);
    if (rc) return rc;
    strtab words;
    count_words(text, n, &sp, &words);
    bbuf ob = {0};
    bb_u32(&ob, (uint32_t)words.n);
    for (size_t i = 0; i < words.n; i++) {
        bb_u32(&ob, words.len[i]);
        bb_put(&ob, st_bytes(&words, i), words.len[i]);
        bb_u64(&ob, (uint64_t)words.val[i]);
    }
    out->data = ob.p; out->n = ob.n;
    st_free(&words); free(sp.p); free(sp.n);
    return OR_OK;
}

static void span_out(void* ctx, size_t start, size_t len) {
    bbuf* b = ctx;
    bb_u64(b, start); bb_u64(b, len);
}
int oracle_pretokenize(const uint8_t* text, size_t n, oracle_blob* out) {
    bbuf ob = {0};
    pretokenize(text, n, span_out, &ob);
    out->data = ob.p; out->n = ob.n;
    return OR_OK;
}

/* ------------------------------------------------------------ encode (tokenizer.py) */
typedef struct {
    strtab tok;              /* byte strings seen (vocab entries, merge parts, products) */
    int64_t* inv;            /* tok id -> vocab id (vocab_inv), -1 if absent */
    size_t inv_cap;
    ptab rank;               /* (tok a, tok b) -> rank (last wins, tokenizer.py:115) */
    uint32_t* prod; size_t prod_cap;  /* rank -> tok id of a+b */
    speclist sp;             /* deduped, sorted longest-first (tokenizer.py:29-30) */
    int has_specials;
    strtab cache;            /* pretoken -> encoded ids (val = offset into cache_ids) */
    bbuf cache_ids;
} encoder;

static void enc_inv_set(encoder* E, size_t tid, int64_t vid) {
    while (E->inv_cap <= tid) {
        size_t nc = E->inv_cap ? E->inv_cap * 2 : 1024;
        E->inv = realloc(E->inv, nc * sizeof(int64_t));
        for (size_t i = E->inv_cap; i < nc; i++) E->inv[i] = -1;
        E->inv_cap = nc;
    }
    E->inv[tid] = vid;
}
static int64_t enc_inv_get(const encoder* E, size_t tid) {
    return tid < E->inv_cap ? E->inv[tid] : -1;
}

/* BPE one pretoken (tokenizer.py:124-136); appends vocab ids to out */
static int enc_word(encoder* E, const uint8_t* p, size_t n, bbuf* out) {
    int64_t hit = st_find(&E->cache, p, n);
    if (hit >= 0) {
        size_t off = (size_t)E->cache.val[hit];
        uint32_t cnt; memcpy(&cnt, E->cache_ids.p + off, 4);
        bb_put(out, E->cache_ids.p + off + 4, (size_t)cnt * 4);
        return OR_OK;
    }
    uint32_t* t = malloc((n ? n : 1) * sizeof(uint32_t));
    size_t len = n;
    for (size_t i = 0; i < n; i++) t[i] = (uint32_t)st_intern(&E->tok, p + i, 1, NULL);
    while (len > 1) {
        int64_t best_rank = -1; size_t best_i = 0;
        for (size_t i = 0; i + 1 < len; i++) {
            pslot* s = pt_get(&E->rank, PKEY(t[i], t[i + 1]), 0);
            if (s && (best_rank < 0 || s->count < best_rank)) { best_rank = s->count; best_i = i; }
        }
        if (best_rank < 0) break;                        /* pair not in inv_merges (130) */
        uint32_t a = t[best_i], b = t[best_i + 1], m = E->prod[best_rank];
        size_t j = 0;                                     /* merge() (92-109) */
        for (size_t i = 0; i < len;) {
            if (t[i] == a && i + 1 < len && t[i + 1] == b) { t[j++] = m; i += 2; }
            else t[j++] = t[i++];
        }
        len = j;
    }
    bbuf ids = {0};
    for (size_t i = 0; i < len; i++) {
        int64_t v = enc_inv_get(E, t[i]);
        if (v < 0) { free(t); free(ids.p); return OR_E_KEY; }   /* vocab_inv[byte] KeyError */
        bb_u32(&ids, (uint32_t)v);
    }
    size_t off = E->cache_ids.n;
    bb_u32(&E->cache_ids, (uint32_t)len);
    bb_put(&E->cache_ids, ids.p, ids.n);
    size_t cid = st_intern(&E->cache, p, n, NULL);
    E->cache.val[cid] = (int64_t)off;
    bb_put(out, ids.p, ids.n);
    free(ids.p); free(t);
    return OR_OK;
}

typedef struct { encoder* E; const uint8_t* seg; bbuf* out; int rc; } encspan_ctx;
static void enc_span(void* vctx, size_t start, size_t len) {
    encspan_ctx* c = vctx;
    if (c->rc) return;
    if (is_special(&c->E->sp, c->seg + start, len)) return;    /* match() drops specials (73) */
    c->rc = enc_word(c->E, c->seg + start, len, c->out);
}

static int enc_segment(encoder* E, const uint8_t* s, size_t n, bbuf* out) {
    if (n == 0) return OR_OK;                                     /* pretokenize (83) */
    if (is_special(&E->sp, s, n)) {                               /* (85-86, 119-122) */
        int64_t tid = st_find(&E->tok, s, n);
        int64_t v = tid >= 0 ? enc_inv_get(E, (size_t)tid) : -1;
        if (v < 0) return OR_E_KEY;
        bb_u32(out, (uint32_t)v);
        return OR_OK;
    }
    encspan_ctx c = {E, s, out, OR_OK};
    pretokenize(s, n, enc_span, &c);
    return c.rc;
}

/* Tokenizer.__init__ (tokenizer.py:12-38) into E; the caller frees it with enc_free */
static int enc_setup(encoder* E, const uint8_t* vocab_blob, size_t vocab_n, const uint8_t* merges_blob,
                     size_t merges_n, const uint8_t* specials_blob, size_t specials_n, speclist* raw) {
    memset(E, 0, sizeof(*E));
    memset(raw, 0, sizeof(*raw));
    st_init(&E->tok, 1 << 12);
    st_init(&E->cache, 1 << 12);
    pt_init(&E->rank);
    /* vocab blob: u32 count, then (i64 id, u32 len, bytes) in dict order; vocab_inv is
     * {v: k for k, v in vocab.items()} -> the last id wins (tokenizer.py:19) */
    uint32_t vc; size_t off = 4;
    if (vocab_n < 4) return OR_E_ARG;
    memcpy(&vc, vocab_blob, 4);
    size_t vsize = 0;
    for (uint32_t i = 0; i < vc; i++) {
        int64_t id; uint32_t l;
        memcpy(&id, vocab_blob + off, 8); off += 8;
        memcpy(&l, vocab_blob + off, 4); off += 4;
        size_t tid = st_intern(&E->tok, vocab_blob + off, l, NULL);
        off += l;
        enc_inv_set(E, tid, id);
        vsize++;
    }
    /* merges blob: u32 count, then (u32 la, a, u32 lb, b) */
    uint32_t mc; off = 4;
    memcpy(&mc, merges_blob, 4);
    E->prod = malloc((mc ? mc : 1) * sizeof(uint32_t));
    for (uint32_t i = 0; i < mc; i++) {
        uint32_t la, lb;
        memcpy(&la, merges_blob + off, 4); off += 4;
        const uint8_t* pa = merges_blob + off; off += la;
        memcpy(&lb, merges_blob + off, 4); off += 4;
        const uint8_t* pb = merges_blob + off; off += lb;
        uint32_t ta = (uint32_t)st_intern(&E->tok, pa, la, NULL);
        uint32_t tb = (uint32_t)st_intern(&E->tok, pb, lb, NULL);
        uint8_t* cat = malloc(la + lb + 1);
        memcpy(cat, pa, la); memcpy(cat + la, pb, lb);
        E->prod[i] = (uint32_t)st_intern(&E->tok, cat, la + lb, NULL);
        free(cat);
        pslot* s = pt_get(&E->rank, PKEY(ta, tb), 1);
        s->count = i;                                     /* later duplicates overwrite */
    }
    /* specials: set() dedupe, then stable sort by length descending (tokenizer.py:29-30);
     * equal-length order only affects ids of missing specials -- we keep input order */
    int rc = parse_specials(specials_blob, specials_n, raw);
    if (rc) return rc;
    E->sp.p = malloc((raw->count + 1) * sizeof(*E->sp.p));
    E->sp.n = malloc((raw->count + 1) * sizeof(*E->sp.n));
    for (size_t i = 0; i < raw->count; i++)
        if (!is_special(&E->sp, raw->p[i], raw->n[i])) {
            E->sp.p[E->sp.count] = raw->p[i]; E->sp.n[E->sp.count] = raw->n[i]; E->sp.count++;
        }
    for (size_t i = 1; i < E->sp.count; i++) {            /* insertion sort, stable */
        const uint8_t* pp = E->sp.p[i]; size_t nn = E->sp.n[i]; size_t j = i;
        while (j > 0 && E->sp.n[j - 1] < nn) { E->sp.p[j] = E->sp.p[j - 1]; E->sp.n[j] = E->sp.n[j - 1]; j--; }
        E->sp.p[j] = pp; E->sp.n[j] = nn;
    }
    /* missing specials get ids len(vocab), len(vocab)+1, ... (tokenizer.py:35-38) */
    size_t next_id = vsize;
    for (size_t i = 0; i < E->sp.count; i++) {
        size_t tid = st_intern(&E->tok, E->sp.p[i], E->sp.n[i], NULL);
        if (enc_inv_get(E, tid) < 0) { enc_inv_set(E, tid, (int64_t)next_id); next_id++; }
    }
    return OR_OK;
}

static void enc_free(encoder* E, speclist* raw) {
    st_free(&E->tok); st_free(&E->cache); free(E->cache_ids.p); free(E->inv);
    free(E->rank.s); free(E->prod); free(E->sp.p); free(E->sp.n); free(raw->p); free(raw->n);
}

/* Tokenizer.encode(text) (tokenizer.py:111-138): segment (63-66: leftmost match, alternatives
 * longest-first), then each segment on its own; ids appended to ob */
static int enc_text(encoder* E, const uint8_t* text, size_t n, bbuf* ob) {
    int rc = OR_OK;
    size_t segstart = 0;
    for (size_t p = 0; p < n && rc == OR_OK;) {
        size_t hit = 0; int found = 0;
        for (size_t k = 0; k < E->sp.count; k++)
            if (E->sp.n[k] > 0 && p + E->sp.n[k] <= n && memcmp(text + p, E->sp.p[k], E->sp.n[k]) == 0) {
                hit = E->sp.n[k]; found = 1; break;
            }
        if (!found) { p++; continue; }
        rc = enc_segment(E, text + segstart, p - segstart, ob);
        if (rc == OR_OK) rc = enc_segment(E, text + p, hit, ob);
        p += hit; segstart = p;
    }
    if (rc == OR_OK) rc = enc_segment(E, text + segstart, n - segstart, ob);
    return rc;
}

int oracle_encode(const uint8_t* vocab_blob, size_t vocab_n, const uint8_t* merges_blob,
                  size_t merges_n, const uint8_t* specials_blob, size_t specials_n,
                  int specials_is_none, const uint8_t* text, size_t n, oracle_blob* out) {
    (void)specials_is_none;
    return oracle_encode_pieces(vocab_blob, vocab_n, merges_blob, merges_n, specials_blob, specials_n,
                                text, n, NULL, 0, out);
}

/* encode.py:31-36: the text read in pieces (f.read(1 M characters)), each piece encoded on its
 * own and the ids concatenated.  starts: sorted byte offsets where pieces begin (0 implied). */
int oracle_encode_pieces(const uint8_t* vocab_blob, size_t vocab_n, const uint8_t* merges_blob,
                         size_t merges_n, const uint8_t* specials_blob, size_t specials_n,
                         const uint8_t* text, size_t n, const uint64_t* starts, size_t n_starts,
                         oracle_blob* out) {
    encoder E; speclist raw;
    out->data = NULL; out->n = 0;
    int rc = enc_setup(&E, vocab_blob, vocab_n, merges_blob, merges_n, specials_blob, specials_n, &raw);
    bbuf ob = {0};
    size_t lo = 0;
    for (size_t i = 0; i <= n_starts && rc == OR_OK; i++) {
        size_t hi = i < n_starts ? (size_t)starts[i] : n;
        if (hi > n) hi = n;
        if (hi < lo) { rc = OR_E_ARG; break; }
        if (hi > lo) rc = enc_text(&E, text + lo, hi - lo, &ob);
        lo = hi;
    }
    enc_free(&E, &raw);
    if (rc) { free(ob.p); return rc; }
    out->data = ob.p; out->n = ob.n;
    return OR_OK;
}

void oracle_free(oracle_blob* b) {
    if (b && b->data) { free(b->data); b->data = NULL; b->n = 0; }
}

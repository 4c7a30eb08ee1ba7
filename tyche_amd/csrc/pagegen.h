/*
 * pagegen.h -- deterministic synthetic page generator, shared by the HIP
 * bench/test kernels and the host (same code compiled for both sides).
 *
 * tyche caches database pages read from disk (io__get_pages, src/io.c:34-80;
 * sample_data/{8k,16k,32k}/names/{tables,indexes}).  The GPU box has no copy
 * of those files, so bench.py and the tests synthesise pages with the same
 * structure: a 24-byte page header, a 4-byte line-pointer array growing up
 * from the header, zeroed free space, and items packed down from the page end
 * (heap tuples with a 24-byte tuple header + short varlena text + ints, or
 * 16-byte btree index tuples over sorted dates).  The mix is tuned so the LZ4
 * 1.7.5 ratio lands at 2.6-2.7 like the sample pages.
 *
 * Every output dword is a pure function of (seed, page index, byte offset),
 * so a GPU thread can fill any dword of any page independently.
 * Page i is keyed by splitmix64(seed ^ i).
 */
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define PG_HD __host__ __device__ __forceinline__
#else
#define PG_HD static inline
#endif

enum {
    PG_DIST_MIX = 0,     /* heap + index pages, the bench default ("pg-heap" mix) */
    PG_DIST_HEAP = 1,
    PG_DIST_INDEX = 2,
    PG_DIST_ZERO = 3,
    PG_DIST_RANDOM = 4,  /* incompressible */
    PG_DIST_TEXT = 5,    /* word salad */
    PG_DIST_COUNT = 6
};

PG_HD uint64_t pg_mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

/* 64 first names, 3..11 letters; packed as 12-byte slots, NUL padded */
#define PG_NAMES 64
#define PG_NAME_SLOT 12
PG_HD const char *pg_name_table() {
    return "Aaliyah\0\0\0\0\0" "Abigail\0\0\0\0\0" "Adeline\0\0\0\0\0" "Alberta\0\0\0\0\0"
           "Alondra\0\0\0\0\0" "Amber\0\0\0\0\0\0\0" "Annabelle\0\0\0" "Antonia\0\0\0\0\0"
           "Aurora\0\0\0\0\0\0" "Beatrice\0\0\0\0" "Bethany\0\0\0\0\0" "Bonnie\0\0\0\0\0\0"
           "Brianna\0\0\0\0\0" "Bridget\0\0\0\0\0" "Camila\0\0\0\0\0\0" "Carmen\0\0\0\0\0\0"
           "Cassandra\0\0\0" "Cecilia\0\0\0\0\0" "Charlotte\0\0\0" "Clara\0\0\0\0\0\0\0"
           "Daisy\0\0\0\0\0\0\0" "Delilah\0\0\0\0\0" "Dolores\0\0\0\0\0" "Eleanor\0\0\0\0\0"
           "Elena\0\0\0\0\0\0\0" "Eloise\0\0\0\0\0\0" "Esther\0\0\0\0\0\0" "Evelyn\0\0\0\0\0\0"
           "Fatima\0\0\0\0\0\0" "Felicity\0\0\0\0" "Florence\0\0\0\0" "Frances\0\0\0\0\0"
           "Gabriela\0\0\0\0" "Genevieve\0\0\0" "Georgia\0\0\0\0\0" "Gloria\0\0\0\0\0\0"
           "Hannah\0\0\0\0\0\0" "Harriet\0\0\0\0\0" "Hazel\0\0\0\0\0\0\0" "Imogen\0\0\0\0\0\0"
           "Ingrid\0\0\0\0\0\0" "Isabella\0\0\0\0" "Ivy\0\0\0\0\0\0\0\0\0" "Jacqueline\0\0"
           "Jasmine\0\0\0\0\0" "Josephine\0\0\0" "Juniper\0\0\0\0\0" "Katherine\0\0\0"
           "Leonora\0\0\0\0\0" "Lucinda\0\0\0\0\0" "Mabel\0\0\0\0\0\0\0" "Marisol\0\0\0\0\0"
           "Matilda\0\0\0\0\0" "Nadia\0\0\0\0\0\0\0" "Octavia\0\0\0\0\0" "Penelope\0\0\0\0"
           "Priscilla\0\0\0" "Rosalind\0\0\0\0" "Savannah\0\0\0\0" "Theodora\0\0\0\0"
           "Ursula\0\0\0\0\0\0" "Valentina\0\0\0" "Winifred\0\0\0\0" "Zenobia\0\0\0\0\0";
}
PG_HD uint32_t pg_name_len(uint32_t id) {
    const char *n = pg_name_table() + id * PG_NAME_SLOT;
    uint32_t l = 0;
    while (l < PG_NAME_SLOT && n[l]) l++;
    return l;
}

#define PG_TEXT_WORDS 32
#define PG_WORD_SLOT 10
PG_HD const char *pg_word_table() {
    return "the\0\0\0\0\0\0\0" "cache\0\0\0\0\0" "page\0\0\0\0\0\0" "buffer\0\0\0\0" "sweep\0\0\0\0\0"
           "clock\0\0\0\0\0" "victim\0\0\0\0" "restore\0\0\0" "pool\0\0\0\0\0\0" "memory\0\0\0\0"
           "raw\0\0\0\0\0\0\0" "ratio\0\0\0\0\0" "hit\0\0\0\0\0\0\0" "list\0\0\0\0\0\0" "of\0\0\0\0\0\0\0\0"
           "and\0\0\0\0\0\0\0" "a\0\0\0\0\0\0\0\0\0" "to\0\0\0\0\0\0\0\0" "in\0\0\0\0\0\0\0\0" "compressed\0"
           "is\0\0\0\0\0\0\0\0" "for\0\0\0\0\0\0\0" "with\0\0\0\0\0\0" "data\0\0\0\0\0\0" "block\0\0\0\0\0"
           "stream\0\0\0\0" "token\0\0\0\0\0" "match\0\0\0\0\0" "offset\0\0\0\0" "length\0\0\0\0"
           "window\0\0\0\0" "table\0\0\0";
}

typedef struct {
    uint64_t key;       /* splitmix64(seed ^ index) */
    uint32_t len;       /* page length in bytes (multiple of 4, >= 64) */
    uint32_t kind;      /* PG_DIST_HEAP .. PG_DIST_TEXT */
    uint32_t nitems;
    uint32_t stride;    /* bytes per item slot */
    uint32_t lower;     /* end of the line-pointer array */
    uint32_t upper;     /* start of the item area */
    uint32_t special;   /* start of the special area (index pages) */
    uint32_t blkno;
} pg_page_t;

PG_HD void pg_page_init(pg_page_t *p, uint64_t seed, uint64_t index, uint32_t len, uint32_t dist) {
    uint64_t k = pg_mix64(seed ^ index);
    p->key = k;
    p->len = len;
    p->blkno = (uint32_t)(index & 0xFFFFFFu);
    uint32_t kind = dist;
    if (dist == PG_DIST_MIX) kind = ((k >> 60) < 13) ? PG_DIST_HEAP : PG_DIST_INDEX;  /* 13/16 heap */
    p->kind = kind;
    p->nitems = 0;
    p->stride = 0;
    p->lower = 24;
    p->upper = len;
    p->special = len;
    if (kind == PG_DIST_HEAP) {
        p->stride = 56;
        uint32_t room = (len - 24) / (p->stride + 4);
        uint32_t fill = 88 + (uint32_t)((k >> 8) % 13);      /* 88..100 % full */
        p->nitems = room * fill / 100;
        if (p->nitems < 1) p->nitems = 1;
    } else if (kind == PG_DIST_INDEX) {
        p->stride = 16;
        p->special = len - 16;
        uint32_t room = (p->special - 24) / (p->stride + 4);
        uint32_t fill = 80 + (uint32_t)((k >> 8) % 21);      /* 80..100 % full */
        p->nitems = room * fill / 100;
        if (p->nitems < 1) p->nitems = 1;
    }
    p->lower = 24 + 4 * p->nitems;
    p->upper = p->special - p->nitems * p->stride;
}

/* per-item hash */
PG_HD uint64_t pg_item_key(const pg_page_t *p, uint32_t item) {
    return pg_mix64(p->key ^ (0x51ED2701u + (uint64_t)item * 0x2545F4914F6CDD1Dull));
}

/* heap tuple image: returns the byte at offset b (< stride) of tuple `item`, and its used length */
PG_HD uint32_t pg_heap_tuple_len(const pg_page_t *p, uint32_t item) {
    uint64_t h = pg_item_key(p, item);
    uint32_t nlen = pg_name_len((uint32_t)(h % PG_NAMES));
    return ((37 + nlen + 3) & ~3u) + 4;
}
PG_HD uint32_t pg_heap_tuple_byte(const pg_page_t *p, uint32_t item, uint32_t b) {
    uint64_t h = pg_item_key(p, item);
    uint32_t name = (uint32_t)(h % PG_NAMES);
    uint32_t nlen = pg_name_len(name);
    uint32_t xmin = 0x2386u + (uint32_t)((p->key >> 20) & 0xFF) * 0x100u + (((h >> 40) & 7) == 0 ? 1u : 0u);
    uint32_t cnt_off = (37 + nlen + 3) & ~3u;
    uint32_t year = ((h >> 12) & 3) == 0 ? 1950 + (uint32_t)((h >> 14) % 60) : 1990 + (uint32_t)((p->key >> 30) % 20);
    uint32_t count = (uint32_t)((h >> 24) & 0x3FFFFu);
    if (b < 4) return (xmin >> (8 * b)) & 0xFF;
    if (b < 12) return 0;                                   /* xmax, cid */
    if (b < 14) return 0;                                   /* ctid block hi */
    if (b < 16) return (p->blkno >> (8 * (b - 14))) & 0xFF; /* ctid block lo */
    if (b < 18) return ((item + 1) >> (8 * (b - 16))) & 0xFF;
    if (b == 18) return 5;                                  /* natts */
    if (b == 19) return 0;
    if (b == 20) return 0x02;
    if (b == 21) return 0x09;
    if (b == 22) return 24;                                 /* t_hoff */
    if (b == 23) return 0;
    if (b == 24) return 0x07;                               /* 'CA' */
    if (b == 25) return ((h >> 50) & 15) == 0 ? 'N' : 'C';
    if (b == 26) return ((h >> 50) & 15) == 0 ? 'Y' : 'A';
    if (b == 27) return 0x05;
    if (b == 28) return ((h >> 55) & 7) == 0 ? 'M' : 'F';
    if (b < 32) return 0;
    if (b < 36) return (year >> (8 * (b - 32))) & 0xFF;
    if (b == 36) return ((nlen + 1) << 1) | 1;
    if (b < 37 + nlen) return (uint8_t)pg_name_table()[name * PG_NAME_SLOT + (b - 37)];
    if (b < cnt_off) return 0;
    if (b < cnt_off + 4) return (count >> (8 * (b - cnt_off))) & 0xFF;
    return 0;
}

PG_HD uint32_t pg_index_tuple_byte(const pg_page_t *p, uint32_t item, uint32_t b) {
    /* btree leaf over a date column: runs of equal keys whose heap pointers walk
     * consecutive line pointers of consecutive heap blocks (sample_data dob_idx) */
    uint32_t run = 12 + (uint32_t)((p->key >> 24) % 40);
    uint32_t base = 6000 + (uint32_t)((p->key >> 16) % 20000);
    uint32_t key = base + item / run;
    uint32_t per_blk = 150 + (uint32_t)((p->key >> 40) % 80);
    uint32_t heapblk = (uint32_t)((p->key >> 8) % 100000) + item / per_blk;
    uint32_t heapoff = per_blk - (item % per_blk);
    if (b < 2) return (heapblk >> (16 + 8 * b)) & 0xFF;
    if (b < 4) return (heapblk >> (8 * (b - 2))) & 0xFF;
    if (b < 6) return (heapoff >> (8 * (b - 4))) & 0xFF;
    if (b == 6) return 16;                                  /* t_info: size */
    if (b == 7) return 0;
    if (b < 12) return (key >> (8 * (b - 8))) & 0xFF;
    return 0;
}

PG_HD uint32_t pg_text_byte(const pg_page_t *p, uint32_t off) {
    /* 64-byte lines of words separated by spaces, '\n' ends a line */
    uint32_t line = off >> 6, col = off & 63;
    if (col == 63) return '\n';
    uint32_t pos = 0, w = 0;
    for (;;) {
        uint64_t h = pg_mix64(p->key ^ ((uint64_t)line << 8 | w));
        uint32_t id = (uint32_t)(h % PG_TEXT_WORDS);
        const char *word = pg_word_table() + id * PG_WORD_SLOT;
        uint32_t wl = 0;
        while (wl < PG_WORD_SLOT && word[wl]) wl++;
        if (col < pos + wl) return (uint8_t)word[col - pos];
        if (col == pos + wl) return ' ';
        pos += wl + 1;
        w++;
    }
}

PG_HD uint32_t pg_page_byte(const pg_page_t *p, uint32_t off) {
    switch (p->kind) {
    case PG_DIST_ZERO: return 0;
    case PG_DIST_RANDOM: return (uint32_t)(pg_mix64(p->key ^ (off >> 3)) >> (8 * (off & 7))) & 0xFF;
    case PG_DIST_TEXT: return pg_text_byte(p, off);
    default: break;
    }
    uint32_t len = p->len;
    if (off < 24) {
        uint32_t d = off >> 2, sh = 8 * (off & 3), v = 0;
        switch (d) {
        case 0: v = (uint32_t)(p->key >> 60); break;                 /* lsn hi */
        case 1: v = (uint32_t)(p->key >> 16); break;                 /* lsn lo */
        case 2: v = (uint32_t)(p->key & 0xFFFF) | (p->kind == PG_DIST_INDEX ? 0u : 0x40000u); break; /* checksum, flags */
        case 3: v = p->lower | (p->upper << 16); break;
        case 4: v = p->special | ((len | 4u) << 16); break;
        default: v = 0; break;
        }
        return (v >> sh) & 0xFF;
    }
    if (off < p->lower) {
        uint32_t item = (off - 24) >> 2, sh = 8 * (off & 3);
        uint32_t ioff = p->special - (item + 1) * p->stride;
        uint32_t ilen = p->kind == PG_DIST_HEAP ? pg_heap_tuple_len(p, item) : 16u;
        uint32_t lp = ioff | (1u << 15) | (ilen << 17);
        return (lp >> sh) & 0xFF;
    }
    if (off < p->upper) return 0;
    if (off < p->special) {
        uint32_t rel = p->special - 1 - off;            /* items are laid down from the end */
        uint32_t item = rel / p->stride;
        uint32_t b = p->stride - 1 - (rel % p->stride);
        return p->kind == PG_DIST_HEAP ? pg_heap_tuple_byte(p, item, b) : pg_index_tuple_byte(p, item, b);
    }
    /* btree special space: prev, next, level, flags */
    {
        uint32_t b = off - p->special;
        uint32_t v = 0;
        if (b < 4) v = p->blkno ? p->blkno - 1 : 0;
        else if (b < 8) v = p->blkno + 1;
        else if (b < 12) v = 0;
        else v = 1;                                      /* BTP_LEAF */
        return (v >> (8 * (b & 3))) & 0xFF;
    }
}

PG_HD uint32_t pg_page_dword(const pg_page_t *p, uint32_t off) {
    return pg_page_byte(p, off) | (pg_page_byte(p, off + 1) << 8) | (pg_page_byte(p, off + 2) << 16) |
           (pg_page_byte(p, off + 3) << 24);
}

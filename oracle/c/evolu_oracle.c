/*
 * evolu_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * A sequential C restatement of the reference's hot path, for parity checks
 * at BASELINE sizes and for the CPU baseline of bench.py.  It follows the
 * reference line by line, with SQLite replaced by hash sets/maps (the same
 * results: the statements are PK / max lookups), and keeps the trie LITERAL
 * (pointer nodes, 3 children, "hash present" bit) -- independent of the GPU
 * engine's leaf-code representation.
 *
 *   timestamp string / parse / hash ...... packages/evolu/src/timestamp.ts:43-55, 87-88
 *   insertIntoMerkleTree ................. packages/evolu/src/merkleTree.ts:8-50
 *   diffMerkleTrees ...................... packages/evolu/src/merkleTree.ts:52-91
 *   applyMessages ........................ packages/evolu/src/applyMessages.ts:26-131
 *   addMessages / getMessages ............ apps/server/src/index.ts:138-202
 *
 * Pinned by tests/test_oracle_c.py against the Python oracle (itself pinned
 * by the reference's snapshots and node-generated vectors).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------ murmur3 (npm murmurhash@2.0.1, v3) */
static uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

uint32_t evo_murmur3(const uint8_t* d, size_t n) {
  uint32_t h = 0, k;
  size_t i = 0;
  for (; i + 4 <= n; i += 4) {
    k = (uint32_t)d[i] | (uint32_t)d[i + 1] << 8 | (uint32_t)d[i + 2] << 16 | (uint32_t)d[i + 3] << 24;
    k *= 0xcc9e2d51u;
    k = rotl(k, 15) * 0x1b873593u;
    h ^= k;
    h = rotl(h, 13) * 5 + 0xe6546b64u;
  }
  k = 0;
  switch (n & 3) {
    case 3: k ^= (uint32_t)d[i + 2] << 16; /* fallthrough */
    case 2: k ^= (uint32_t)d[i + 1] << 8;  /* fallthrough */
    case 1:
      k ^= d[i];
      k *= 0xcc9e2d51u;
      k = rotl(k, 15) * 0x1b873593u;
      h ^= k;
  }
  h ^= (uint32_t)n;
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

/* ------------------------------------------------------------ dates (Date.parse / toISOString, canonical subset) */
static int64_t days_from_civil(int64_t y, int m, int d) {
  y -= m <= 2;
  int64_t era = (y >= 0 ? y : y - 399) / 400;
  int64_t yoe = y - era * 400;
  int64_t doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + doe - 719468;
}

static int dim(int y, int m) {
  static const int t[] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  if (m == 2 && ((y % 4 == 0 && y % 100 != 0) || y % 400 == 0)) return 29;
  return t[m - 1];
}

static int num(const char* s, int n, int* out) {
  int v = 0;
  for (int i = 0; i < n; ++i) {
    if (s[i] < '0' || s[i] > '9') return 0;
    v = v * 10 + (s[i] - '0');
  }
  *out = v;
  return 1;
}

/* Strict parse of a canonical timestamp (s == toString(fromString(s))),
 * restricted to the engine's native domain: 1970 <= t < 2^31 minutes.
 * Returns 1 and millis/counter, else 0. */
int evo_parse(const char* s, int64_t* millis, int* counter) {
  int y, mo, d, hh, mi, ss, ms;
  if (!num(s, 4, &y) || s[4] != '-' || !num(s + 5, 2, &mo) || s[7] != '-' || !num(s + 8, 2, &d) || s[10] != 'T' ||
      !num(s + 11, 2, &hh) || s[13] != ':' || !num(s + 14, 2, &mi) || s[16] != ':' || !num(s + 17, 2, &ss) ||
      s[19] != '.' || !num(s + 20, 3, &ms) || s[23] != 'Z' || s[24] != '-' || s[29] != '-')
    return 0;
  if (mo < 1 || mo > 12 || d < 1 || d > dim(y, mo) || hh > 23 || mi > 59 || ss > 59) return 0;
  int c = 0;
  for (int i = 25; i < 29; ++i) {
    char ch = s[i];
    int v = ch >= '0' && ch <= '9' ? ch - '0' : ch >= 'A' && ch <= 'F' ? ch - 'A' + 10 : -1;
    if (v < 0) return 0;
    c = c * 16 + v;
  }
  for (int i = 30; i < 46; ++i) {
    char ch = s[i];
    if (!((ch >= '0' && ch <= '9') || (ch >= 'a' && ch <= 'f') || (ch >= 'A' && ch <= 'F'))) return 0;
  }
  if (y < 1970) return 0;
  int64_t m = ((days_from_civil(y, mo, d) * 24 + hh) * 60 + mi) * 60000 + (int64_t)ss * 1000 + ms;
  if (m >= (int64_t)2147483648LL * 60000) return 0;
  *millis = m;
  *counter = c;
  return 1;
}

/* ------------------------------------------------------------ literal trie (merkleTree.ts) */
typedef struct Node {
  struct Node* ch[3];
  int32_t hash;
  int has_hash;
} Node;

static Node* node_new(void) { return (Node*)calloc(1, sizeof(Node)); }
static void node_free(Node* n) {
  if (!n) return;
  for (int i = 0; i < 3; ++i) node_free(n->ch[i]);
  free(n);
}

/* merkleTree.ts:31-50: key = ((millis/1000/60)|0).toString(3); root ^= h; every
 * prefix node ^= h (created on first touch, never removed). */
static void trie_insert(Node* root, int64_t millis, uint32_t h) {
  int32_t minute = (int32_t)(millis / 60000); /* == (millis/1000/60)|0 on the native domain */
  char key[24];
  int len = 0;
  if (minute == 0) key[len++] = '0';
  while (minute > 0) {
    key[len++] = (char)('0' + minute % 3);
    minute /= 3;
  }
  root->hash ^= (int32_t)h;
  root->has_hash = 1;
  Node* n = root;
  for (int i = len - 1; i >= 0; --i) {
    int c = key[i] - '0';
    if (!n->ch[c]) n->ch[c] = node_new();
    n = n->ch[c];
    n->hash ^= (int32_t)h;
    n->has_hash = 1;
  }
}

static void emit(const Node* n, char** buf, size_t* len, size_t* cap) {
  char tmp[40];
  int first = 1;
#define PUT(s)                                  \
  do {                                          \
    size_t l_ = strlen(s);                      \
    if (*len + l_ + 1 > *cap) {                 \
      *cap = (*cap + l_ + 1) * 2;               \
      *buf = (char*)realloc(*buf, *cap);        \
    }                                           \
    memcpy(*buf + *len, s, l_);                 \
    *len += l_;                                 \
  } while (0)
  PUT("{");
  for (int c = 0; c < 3; ++c)
    if (n->ch[c]) {
      snprintf(tmp, sizeof tmp, "%s\"%d\":", first ? "" : ",", c);
      PUT(tmp);
      first = 0;
      emit(n->ch[c], buf, len, cap);
    }
  if (n->has_hash) {
    snprintf(tmp, sizeof tmp, "%s\"hash\":%d", first ? "" : ",", n->hash);
    PUT(tmp);
  }
  PUT("}");
#undef PUT
}

/* merkleTree.ts:63-91, literal greedy descent.  Returns 0 none, 1 some (*out), 2 RangeError */
static int trie_diff(const Node* a, const Node* b, int64_t* out) {
  int ah = a && a->has_hash, bh = b && b->has_hash;
  if (ah == bh && (!ah || a->hash == b->hash)) return 0;
  char k[32];
  int kl = 0;
  for (;;) {
    int pick = -1;
    for (int c = 0; c < 3; ++c) {
      const Node* x = a ? a->ch[c] : NULL;
      const Node* y = b ? b->ch[c] : NULL;
      if (!x && !y) continue;
      int xh = x && x->has_hash, yh = y && y->has_hash;
      if (xh != yh || (xh && x->hash != y->hash)) {
        pick = c;
        break;
      }
    }
    if (pick < 0) break;
    if (kl < 31) k[kl] = (char)('0' + pick);
    ++kl;
    a = a ? a->ch[pick] : NULL;
    b = b ? b->ch[pick] : NULL;
  }
  if (kl > 16) return 2;
  int64_t v = 0;
  for (int i = 0; i < 16; ++i) v = v * 3 + (i < kl ? k[i] - '0' : 0);
  *out = v * 60000;
  return 1;
}

/* ------------------------------------------------------------ string hash set / map (open addressing) */
typedef struct {
  const char** key; /* 46-byte strings (not owned) */
  int32_t* val;
  uint64_t* tag;
  size_t cap;
  size_t n;
} Map;

static uint64_t fnv(const char* s, size_t n, uint64_t salt) {
  uint64_t h = 1469598103934665603ull ^ salt;
  for (size_t i = 0; i < n; ++i) h = (h ^ (uint8_t)s[i]) * 1099511628211ull;
  return h | 1;
}

static void map_init(Map* m, size_t cap) {
  size_t c = 16;
  while (c < cap * 2) c <<= 1;
  m->cap = c;
  m->n = 0;
  m->key = (const char**)calloc(c, sizeof(char*));
  m->val = (int32_t*)calloc(c, sizeof(int32_t));
  m->tag = (uint64_t*)calloc(c, sizeof(uint64_t));
}
static void map_free(Map* m) {
  free(m->key);
  free(m->val);
  free(m->tag);
}
/* slot for (s, salt); *found set if present */
static size_t map_slot(Map* m, const char* s, size_t n, uint64_t salt, int* found) {
  uint64_t t = fnv(s, n, salt);
  size_t p = t & (m->cap - 1);
  for (;;) {
    if (!m->tag[p]) {
      *found = 0;
      return p;
    }
    if (m->tag[p] == t && memcmp(m->key[p], s, n) == 0) {
      *found = 1;
      return p;
    }
    p = (p + 1) & (m->cap - 1);
  }
}

/* ------------------------------------------------------------ applyMessages (one owner) */
/* Inputs: n timestamps at `stride`, cell ids (dense), prior per-cell max
 * timestamps (prior_present[c] ? prior + c*pstride : none).  Outputs: flags
 * (1 ups | 2 xor), winner per cell, and the tree JSON (caller frees with
 * evo_free).  Returns 0 ok, 2 non-canonical, 3 cross-cell PK collision. */
int evo_apply(const char* ts, size_t stride, size_t n, const uint32_t* cell, uint32_t n_cells, const char* prior,
              size_t pstride, const uint8_t* prior_present, uint8_t* flags, int32_t* winner, char** json) {
  const char** cur = (const char**)calloc(n_cells ? n_cells : 1, sizeof(char*)); /* current max per cell */
  Map pk; /* __message PRIMARY KEY: timestamp -> cell */
  map_init(&pk, n + n_cells + 1);
  Node* root = node_new();
  int status = 0;
  for (uint32_t c = 0; c < n_cells; ++c) {
    winner[c] = -1;
    if (prior_present && prior_present[c]) {
      cur[c] = prior + (size_t)c * pstride;
      int f;
      size_t p = map_slot(&pk, cur[c], 46, 0, &f);
      if (!f) {
        pk.tag[p] = fnv(cur[c], 46, 0);
        pk.key[p] = cur[c];
        pk.val[p] = (int32_t)c;
      }
    }
  }
  for (size_t i = 0; i < n && !status; ++i) {
    const char* s = ts + i * stride;
    const uint32_t c = cell[i];
    int64_t millis;
    int counter;
    if (!evo_parse(s, &millis, &counter)) {
      status = 2;
      break;
    }
    const char* t = cur[c];                      /* SELECT ... ORDER BY timestamp DESC LIMIT 1 */
    const int cmp = t ? memcmp(t, s, 46) : -1;   /* JS string compare == byte compare (ASCII) */
    const int ups = !t || cmp < 0;               /* applyMessages.ts:93 */
    const int xr = !t || cmp != 0;               /* applyMessages.ts:105 */
    flags[i] = (uint8_t)((ups ? 1 : 0) | (xr ? 2 : 0));
    if (ups) winner[c] = (int32_t)i;
    if (xr) {
      int f;
      size_t p = map_slot(&pk, s, 46, 0, &f);
      if (!f) { /* INSERT took: the cell's max may move */
        pk.tag[p] = fnv(s, 46, 0);
        pk.key[p] = s;
        pk.val[p] = (int32_t)c;
        if (!t || cmp < 0) cur[c] = s;
      } else if ((uint32_t)pk.val[p] != c) {
        status = 3; /* the engine reports this case instead of modelling it */
      }
      trie_insert(root, millis, evo_murmur3((const uint8_t*)s, 46));
    }
  }
  if (!status && json) {
    size_t len = 0, cap = 256;
    *json = (char*)malloc(cap);
    emit(root, json, &len, &cap);
    (*json)[len] = 0;
  }
  node_free(root);
  map_free(&pk);
  free(cur);
  return status;
}

/* ------------------------------------------------------------ server (index.ts) */
/* One batch for many owners; trees persist across calls in a Server object. */
typedef struct {
  uint32_t n_owners;
  Node** tree;
  Map rows; /* (timestamp, owner) */
  char** arena;
  size_t n_arena;
} Server;

void* evo_server_new(uint32_t n_owners, size_t cap) {
  Server* s = (Server*)calloc(1, sizeof(Server));
  s->n_owners = n_owners;
  s->tree = (Node**)calloc(n_owners ? n_owners : 1, sizeof(Node*));
  for (uint32_t o = 0; o < n_owners; ++o) s->tree[o] = node_new();
  map_init(&s->rows, cap + 1);
  return s;
}

void evo_server_free(void* p) {
  Server* s = (Server*)p;
  for (uint32_t o = 0; o < s->n_owners; ++o) node_free(s->tree[o]);
  free(s->tree);
  map_free(&s->rows);
  for (size_t i = 0; i < s->n_arena; ++i) free(s->arena[i]);
  free(s->arena);
  free(s);
}

/* index.ts:138-171 in batch order; flags[i] = 4 iff the row was inserted */
int evo_server_ingest(void* p, const char* ts, size_t stride, size_t n, const uint32_t* owner, uint8_t* flags) {
  Server* s = (Server*)p;
  /* PRIMARY KEY(timestamp, userId): the map key is the 46 bytes + the owner */
  char* copy = (char*)malloc(n * 50 + 1);
  s->arena = (char**)realloc(s->arena, sizeof(char*) * (s->n_arena + 1));
  s->arena[s->n_arena++] = copy;
  for (size_t i = 0; i < n; ++i) {
    const char* t = ts + i * stride;
    int64_t millis;
    int counter;
    if (!evo_parse(t, &millis, &counter)) return 2;
    char* k = copy + i * 50;
    memcpy(k, t, 46);
    memcpy(k + 46, &owner[i], 4);
    int f;
    size_t q = map_slot(&s->rows, k, 50, 0, &f);
    flags[i] = f ? 0 : 4; /* INSERT OR IGNORE: changes === 1 */
    if (!f) {
      if (s->rows.n * 2 + 2 > s->rows.cap) return 8; /* capacity */
      s->rows.tag[q] = fnv(k, 50, 0);
      s->rows.key[q] = k;
      s->rows.n++;
      trie_insert(s->tree[owner[i]], millis, evo_murmur3((const uint8_t*)t, 46));
    }
  }
  return 0;
}

char* evo_server_tree_json(void* p, uint32_t owner) {
  Server* s = (Server*)p;
  size_t len = 0, cap = 256;
  char* out = (char*)malloc(cap);
  emit(s->tree[owner], &out, &len, &cap);
  out[len] = 0;
  return out;
}

/* diff of two servers' trees for one owner (the "client" is another Server) */
int evo_server_diff(void* a, void* b, uint32_t owner, int64_t* millis) {
  return trie_diff(((Server*)a)->tree[owner], ((Server*)b)->tree[owner], millis);
}

/* merkleTree.ts:31-50 over a list: JSON of the tree of n timestamps */
char* evo_tree_json(const char* ts, size_t stride, size_t n) {
  Node* root = node_new();
  for (size_t i = 0; i < n; ++i) {
    int64_t m;
    int c;
    if (evo_parse(ts + i * stride, &m, &c)) trie_insert(root, m, evo_murmur3((const uint8_t*)(ts + i * stride), 46));
  }
  size_t len = 0, cap = 256;
  char* out = (char*)malloc(cap);
  emit(root, &out, &len, &cap);
  out[len] = 0;
  node_free(root);
  return out;
}

void evo_free(void* p) { free(p); }

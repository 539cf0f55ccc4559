// g2048_core.h -- bitboard arithmetic of the 2048 hot path, shared by the gfx950 kernels (g2048.hip) and the
// CPU unit-test harness (tests/native/core_test.cpp, test-only).  Nothing here allocates or launches.
//
// Board ("bitboard"): uint64, nibble i = 4*r + c holds log2(tile) (0 = empty); row r = bits [16r, 16r+16),
// cell c = nibble c of its row.  A "line" is 4 nibbles in move-left frame order (nibble 0 = destination edge).
//
// Every function names the reference semantics it implements (paths relative to the reference repo root).
#pragma once
#include <math.h>
#include <stdint.h>

#ifdef __HIPCC__
#define G2048_HD __host__ __device__ inline
#else
#define G2048_HD static inline  // test-only host build of the same code
#endif

namespace g2048 {

constexpr uint64_t kNibLsb = 0x1111111111111111ull;
constexpr uint64_t kHMask = 0x0111011101110111ull;  // cells with c in {0,1,2}: a right-hand neighbour exists
constexpr uint64_t kVMask = 0x0000111111111111ull;  // cells with r in {0,1,2}: a lower neighbour exists

G2048_HD int popc64(uint64_t x) { return __builtin_popcountll(x); }

// bit 4i set iff nibble i != 0
G2048_HD uint64_t nz_bits(uint64_t b) {
    uint64_t x = b | (b >> 1);
    x |= x >> 2;
    return x & kNibLsb;
}

// 4x4 nibble transpose: cell (r,c) <-> (c,r)
G2048_HD uint64_t transpose(uint64_t x) {
    uint64_t t = (x ^ (x >> 12)) & 0x0000F0F00000F0F0ull;
    x ^= t ^ (t << 12);
    t = (x ^ (x >> 24)) & 0x00000000FF00FF00ull;
    x ^= t ^ (t << 24);
    return x;
}

// reverse the 4 nibbles of every row: cell (r,c) -> (r,3-c)
G2048_HD uint64_t reverse_rows(uint64_t x) {
    x = ((x & 0x00FF00FF00FF00FFull) << 8) | ((x >> 8) & 0x00FF00FF00FF00FFull);
    x = ((x & 0x0F0F0F0F0F0F0F0Full) << 4) | ((x >> 4) & 0x0F0F0F0F0F0F0F0Full);
    return x;
}

// reverse the order of the rows: cell (r,c) -> (3-r,c)
G2048_HD uint64_t reverse_cols(uint64_t x) {
    x = ((x & 0x00000000FFFFFFFFull) << 32) | (x >> 32);
    x = ((x & 0x0000FFFF0000FFFFull) << 16) | ((x >> 16) & 0x0000FFFF0000FFFFull);
    return x;
}

// Game2048._is_done (src/game2048.py:172-187): no empty cell and no equal horizontal / vertical neighbours.
G2048_HD bool is_done(uint64_t b) {
    uint64_t nz = nz_bits(b);
    if (nz != kNibLsb) return false;
    uint64_t eqh = ~nz_bits(b ^ (b >> 4)) & kHMask;
    uint64_t eqv = ~nz_bits(b ^ (b >> 16)) & kVMask;
    return (eqh | eqv) == 0;
}

// Game2048.get_action_mask (src/game2048.py:95-99, :233-237): bit a set iff action a changes the board.
// A line changes under move-left iff an empty cell precedes a tile or two adjacent tiles are equal.
G2048_HD uint32_t action_mask(uint64_t b) {
    uint64_t nz = nz_bits(b);
    uint64_t z = ~nz & kNibLsb;
    uint64_t eqh = ~nz_bits(b ^ (b >> 4)) & nz & kHMask;
    uint64_t eqv = ~nz_bits(b ^ (b >> 16)) & nz & kVMask;
    uint32_t up = ((z & (nz >> 16) & kVMask) | eqv) != 0;
    uint32_t down = ((nz & (z >> 16) & kVMask) | eqv) != 0;
    uint32_t left = ((z & (nz >> 4) & kHMask) | eqh) != 0;
    uint32_t right = ((nz & (z >> 4) & kHMask) | eqh) != 0;
    return up | (right << 1) | (down << 2) | (left << 3);
}

G2048_HD uint32_t nibble_sum16(uint32_t x) {
    x = (x & 0x0F0Fu) + ((x >> 4) & 0x0F0Fu);
    return (x & 0xFFu) + (x >> 8);
}

// _row_move_left (src/game2048.py:120-137) on one line: compress, merge equal neighbours once left to right,
// compress.  A 15+15 merge saturates at 15 (the caller flags it).  Used to build the row table.
G2048_HD uint32_t line_move_left(uint32_t row) {
    uint32_t c[4];
    int n = 0;
    for (int k = 0; k < 4; k++) {
        uint32_t e = (row >> (4 * k)) & 15u;
        if (e) c[n++] = e;
    }
    uint32_t out = 0;
    int w = 0, i = 0;
    while (i < n) {
        uint32_t e;
        if (i + 1 < n && c[i] == c[i + 1]) {
            e = c[i] + 1;
            if (e > 15) e = 15;
            i += 2;
        } else {
            e = c[i];
            i += 1;
        }
        out |= e << (4 * w);
        w++;
    }
    return out;
}

// What the merges of one line were, recovered from the old and new line (no second table needed):
//   c = tiles(old) - tiles(new) merges; c == 1: merged exponent = sum(old) - sum(new) + 2 (17 => saturated
//   15+15, true exponent 16); c == 2: old was [a,a,b,b] (all four cells full) -> exponents a+1, b+1 in order.
struct LineMerges {
    uint32_t n;       // 0..2
    uint32_t e0, e1;  // merged exponents in list order (true value, up to 16)
};

G2048_HD LineMerges line_merges(uint32_t o, uint32_t nw) {
    LineMerges m;
    uint32_t to = (uint32_t)popc64(nz_bits(o));
    uint32_t tn = (uint32_t)popc64(nz_bits(nw));
    m.n = to - tn;
    uint32_t d = nibble_sum16(o) - nibble_sum16(nw) + 2u;
    uint32_t e_single = d > 16u ? 16u : d;
    uint32_t a = (o & 15u) + 1u, b = ((o >> 8) & 15u) + 1u;
    m.e0 = m.n == 2 ? a : (m.n == 1 ? e_single : 0u);
    m.e1 = m.n == 2 ? b : 0u;
    return m;
}

// 4-bit merge code of a line (second row table, so the kernel need not re-derive merges arithmetically):
//   0 no merge; 1..3 one merge, its result at output position code-1; 4 two merges (results at positions 0, 1);
//   5..7 one merge at position code-5 that saturated (15+15: true exponent 16);
//   8 two merges, first saturated; 9 two merges, second saturated; 10 two merges, both saturated.
G2048_HD uint32_t line_merge_code(uint32_t row) {
    uint32_t c[4];
    int n = 0;
    for (int k = 0; k < 4; k++) {
        uint32_t e = (row >> (4 * k)) & 15u;
        if (e) c[n++] = e;
    }
    int w = 0, i = 0, np = 0;
    int pos[2] = {0, 0};
    bool sat[2] = {false, false};
    while (i < n) {
        if (i + 1 < n && c[i] == c[i + 1]) {
            pos[np] = w;
            sat[np] = c[i] == 15u;
            np++;
            i += 2;
        } else {
            i += 1;
        }
        w++;
    }
    if (np == 0) return 0u;
    if (np == 1) return (uint32_t)(sat[0] ? 5 + pos[0] : 1 + pos[0]);
    return sat[0] ? (sat[1] ? 10u : 8u) : (sat[1] ? 9u : 4u);
}

// Accumulated merge summary of one move (what _compute_reward and Game2048.score consume).
struct MoveSummary {
    uint32_t count;   // len(merged)
    uint32_t sum_e;   // sum(log2(v) for v in merged)  (reward_mode "log2")
    uint32_t score;   // sum(merged)                   (reward_mode "sum", Game2048.score)
    uint32_t max_e;   // log2(max(merged, default=0)) (0 if none)
    uint32_t list;    // merged list, nibble k = e_k - 1, list order
    uint32_t overflow;
};

G2048_HD void summary_add(MoveSummary& s, uint32_t e) {
    // caller guarantees e != 0
    s.list |= ((e - 1u) & 15u) << (4u * (s.count & 7u));
    s.count += 1u;
    s.sum_e += e;
    s.score += 1u << e;
    s.max_e = e > s.max_e ? e : s.max_e;
    s.overflow |= (e >= 16u);
}

// Game2048._move (src/game2048.py:158-165) for action a given a line table `lut` (move-left of each 16-bit
// line).  The reference rotates clockwise (3 - a) times and moves left; here the lines of the move-left frame
// are read directly: left = rows, right = rows reversed, up = columns, down = columns reversed.  The merged
// list follows the reference's row order in the rotated frame: left rows 0..3, right rows 3..0,
// up columns 3..0, down columns 0..3 (each line in frame order).
template <class Lut>
G2048_HD uint64_t board_move(uint64_t b, uint32_t a, const Lut& lut, MoveSummary& s) {
    const bool vert = (a == 0u) | (a == 2u);
    const bool rev = (a == 1u) | (a == 2u);
    const bool back = (a == 0u) | (a == 1u);  // list order runs from line 3 down to line 0
    uint64_t f = vert ? transpose(b) : b;
    f = rev ? reverse_rows(f) : f;
    uint64_t g = 0;
    s.count = s.sum_e = s.score = s.max_e = s.list = s.overflow = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int line = back ? 3 - j : j;
        uint32_t o = (uint32_t)(f >> (16 * line)) & 0xFFFFu;
        uint32_t nw = (uint32_t)lut(o);
        g |= (uint64_t)nw << (16 * line);
        LineMerges m = line_merges(o, nw);
        if (m.n >= 1u) summary_add(s, m.e0);
        if (m.n == 2u) summary_add(s, m.e1);
    }
    g = rev ? reverse_rows(g) : g;
    g = vert ? transpose(g) : g;
    return g;
}

// Branch-free decode of line_merge_code: three constants with two bits per code c (at bit 2c).
//   kDecA: slot-0 kind (0 none, 1 result in the new line at cell kDecP, 2 saturated = exponent 16)
//   kDecB: slot-1 kind (0 none, 1 result at cell 1, 2 saturated)
constexpr uint32_t dec_pack(const uint32_t (&v)[11]) {
    uint32_t r = 0;
    for (int c = 0; c < 11; c++) r |= v[c] << (2 * c);
    return r;
}
constexpr uint32_t kDecAv[11] = {0, 1, 1, 1, 1, 2, 2, 2, 2, 1, 2};
constexpr uint32_t kDecPv[11] = {0, 0, 1, 2, 0, 0, 0, 0, 0, 0, 0};
constexpr uint32_t kDecBv[11] = {0, 0, 0, 0, 1, 0, 0, 0, 1, 2, 2};
constexpr uint32_t kDecA = dec_pack(kDecAv), kDecP = dec_pack(kDecPv), kDecB = dec_pack(kDecBv);

G2048_HD uint32_t bfe32(uint32_t x, uint32_t off, uint32_t w) {
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_amdgcn_ubfe(x, off, w);
#else
    return (x >> off) & ((1u << w) - 1u);
#endif
}

// merged exponents of one line (list order; 16 = saturated 15+15) from its new line and merge code
G2048_HD void decode_merge_code(uint32_t code, uint32_t nw, uint32_t& e0, uint32_t& e1) {
    const uint32_t sh = 2u * code;
    const uint32_t ka = bfe32(kDecA, sh, 2), kb = bfe32(kDecB, sh, 2), p = bfe32(kDecP, sh, 2);
    e0 = (ka == 1u ? bfe32(nw, 4u * p, 4) : 0u) | ((ka & 2u) << 3);
    e1 = (kb == 1u ? bfe32(nw, 4u, 4) : 0u) | ((kb & 2u) << 3);
}

// Board move with the two row tables (`lut(o)` -> new line, `code(o)` -> line_merge_code).  Same result and
// merged-list order as board_move.  Straight-line code (no per-lane branches, so a wave whose lanes hold all
// four actions runs it once): the frame transforms are computed and mask-selected, all eight table reads
// are issued before any is used, the merge summary is accumulated arithmetically (the list only if wanted).
template <bool WANT_LIST, class Lut, class Code>
G2048_HD uint64_t board_move_coded(uint64_t b, uint32_t a, const Lut& lut, const Code& code, MoveSummary& s) {
    const uint64_t mvert = 0ull - (uint64_t)((a == 0u) | (a == 2u));
    const uint64_t mrev = 0ull - (uint64_t)((a == 1u) | (a == 2u));
    const bool back = (a == 0u) | (a == 1u);
    uint64_t f = b ^ ((b ^ transpose(b)) & mvert);
    f ^= (f ^ reverse_rows(f)) & mrev;
    uint32_t o[4], nw[4], c[4];
#pragma unroll
    for (int j = 0; j < 4; j++) o[j] = (uint32_t)(f >> (16 * j)) & 0xFFFFu;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        nw[j] = (uint32_t)lut(o[j]);
        c[j] = (uint32_t)code(o[j]);
    }
    uint64_t g = 0;
    uint32_t sum_e = 0, score = 0, max_e = 0, count = 0, list = 0;
#pragma unroll
    for (int jj = 0; jj < 4; jj++) {
        const int j = jj;
        g |= (uint64_t)nw[j] << (16 * j);
        uint32_t e0, e1;
        decode_merge_code(c[j], nw[j], e0, e1);
        score += ((1u << e0) & ~1u) + ((1u << e1) & ~1u);
        sum_e += e0 + e1;
        max_e = max_e > e0 ? max_e : e0;
        max_e = max_e > e1 ? max_e : e1;
    }
    if (WANT_LIST) {
        // list order: lines 0..3 of the frame, or 3..0 for left/up (the reference's rotated-frame row order)
#pragma unroll
        for (int jj = 0; jj < 4; jj++) {
            const int j0 = jj, j1 = 3 - jj;
            const uint32_t cc = back ? c[j1] : c[j0];
            const uint32_t nn = back ? nw[j1] : nw[j0];
            uint32_t e0, e1;
            decode_merge_code(cc, nn, e0, e1);
            const uint32_t n0 = e0 != 0u, n1 = e1 != 0u;
            if (n0) list |= ((e0 - 1u) & 15u) << (4u * (count & 7u));
            if (n1) list |= ((e1 - 1u) & 15u) << (4u * ((count + n0) & 7u));
            count += n0 + n1;
        }
    } else {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            uint32_t e0, e1;
            decode_merge_code(c[j], nw[j], e0, e1);
            count += (e0 != 0u) + (e1 != 0u);
        }
    }
    s.count = count;
    s.sum_e = sum_e;
    s.score = score;
    s.max_e = max_e;
    s.overflow = max_e >> 4;
    s.list = list;
    g ^= (g ^ reverse_rows(g)) & mrev;
    g ^= (g ^ transpose(g)) & mvert;
    return g;
}

// _row_move_left (src/game2048.py:120-137) of one line without a table: one left-to-right pass holding the pending
// (not yet placed) tile, which either merges with the next equal tile or is placed at the write position.  Returns
// the new line (a 15+15 merge saturates at 15); e0 / e1 = the merged exponents in position order (16 = saturated).
G2048_HD uint32_t line_move_alu(uint32_t o, uint32_t& e0, uint32_t& e1) {
    uint32_t out = 0u, sh = 0u, pend = o & 15u;
    e0 = 0u;
    e1 = 0u;
#pragma unroll
    for (int k = 1; k < 4; k++) {
        const uint32_t v = bfe32(o, 4u * k, 4u);
        const bool nz = v != 0u;
        const bool mg = nz && v == pend;
        const uint32_t emit = mg ? (v == 15u ? 15u : v + 1u) : (nz ? pend : 0u);
        out |= emit << sh;
        sh += emit != 0u ? 4u : 0u;
        e1 = (mg && e0 != 0u) ? v + 1u : e1;
        e0 = (mg && e0 == 0u) ? v + 1u : e0;
        pend = mg ? 0u : (nz ? v : pend);
    }
    return out | (pend << sh);
}

// Game2048._move (src/game2048.py:158-165) with line_move_alu: the same result, summary and merged-list order as
// board_move_coded, and no table (no LDS, no table fill).
template <bool WANT_LIST>
G2048_HD uint64_t board_move_alu(uint64_t b, uint32_t a, MoveSummary& s) {
    const uint64_t mvert = 0ull - (uint64_t)((a == 0u) | (a == 2u));
    const uint64_t mrev = 0ull - (uint64_t)((a == 1u) | (a == 2u));
    const bool back = (a == 0u) | (a == 1u);
    uint64_t f = b ^ ((b ^ transpose(b)) & mvert);
    f ^= (f ^ reverse_rows(f)) & mrev;
    uint32_t e0[4], e1[4];
    uint64_t g = 0;
    uint32_t sum_e = 0, score = 0, max_e = 0, count = 0, list = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t nw = line_move_alu((uint32_t)(f >> (16 * j)) & 0xFFFFu, e0[j], e1[j]);
        g |= (uint64_t)nw << (16 * j);
        score += ((1u << e0[j]) & ~1u) + ((1u << e1[j]) & ~1u);
        sum_e += e0[j] + e1[j];
        max_e = max_e > e0[j] ? max_e : e0[j];
        max_e = max_e > e1[j] ? max_e : e1[j];
    }
    if (WANT_LIST) {
#pragma unroll
        for (int jj = 0; jj < 4; jj++) {
            const uint32_t x0 = back ? e0[3 - jj] : e0[jj], x1 = back ? e1[3 - jj] : e1[jj];
            const uint32_t n0 = x0 != 0u, n1 = x1 != 0u;
            if (n0) list |= ((x0 - 1u) & 15u) << (4u * (count & 7u));
            if (n1) list |= ((x1 - 1u) & 15u) << (4u * ((count + n0) & 7u));
            count += n0 + n1;
        }
    } else {
#pragma unroll
        for (int j = 0; j < 4; j++) count += (e0[j] != 0u) + (e1[j] != 0u);
    }
    s.count = count;
    s.sum_e = sum_e;
    s.score = score;
    s.max_e = max_e;
    s.overflow = max_e >> 4;
    s.list = list;
    g ^= (g ^ reverse_rows(g)) & mrev;
    g ^= (g ^ transpose(g)) & mvert;
    return g;
}

// ---------------------------------------------------------------------------------------------------------
// Lean merge summary (the step kernel's log2-reward path).  The second row table holds, instead of the merge
// code, one 4-bit field per line: 0 = no merge, else (largest merged exponent - 1), 1..15 (15 = a saturated
// 15+15 merge, true exponent 16).  The rest of the summary comes from board aggregates: a merge of two x-tiles
// leaves one (x+1)-tile and touches no other cell, so
//   count = tiles(b) - tiles(g)   and   sum_e = sum(e) = nibsum(b) - nibsum(g) + 2 count
// (each merge removes 2x and adds x+1 = e: nibsum drops by e - 2).  A saturated merge (15+15 -> 15) breaks the
// second identity by 1, so a line field of 15 sends the lane to the exact per-line sum (line_merges).
// ---------------------------------------------------------------------------------------------------------
G2048_HD uint32_t line_max_merge_field(uint32_t row) {
    uint32_t e0, e1;
    (void)line_move_alu(row, e0, e1);  // merged exponents in position order, 16 = saturated
    const uint32_t m = e0 > e1 ? e0 : e1;
    return m ? m - 1u : 0u;            // merged exponents are >= 2, so 0 is free for "no merge"
}

// sum of the 16 nibbles of a board (<= 240)
G2048_HD uint32_t nib_sum64(uint64_t x) {
    const uint64_t t = (x & 0x0F0F0F0F0F0F0F0Full) + ((x >> 4) & 0x0F0F0F0F0F0F0F0Full);  // 8 bytes, each <= 30
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_amdgcn_sad_u8((uint32_t)t, 0u, __builtin_amdgcn_sad_u8((uint32_t)(t >> 32), 0u, 0u));
#else
    uint64_t y = t + (t >> 8);
    y += y >> 16;
    y += y >> 32;
    return (uint32_t)(y & 0xFFu);
#endif
}

// Game2048._move (src/game2048.py:158-165) with the line table and the max-merge field table (`mx`): the same
// board as board_move_coded and the summary fields the log2 reward and max_tile_seen read -- count, sum_e,
// max_e, overflow -- not score or the merged list.  nzg = nz_bits of the moved board (the spawn's empty cells).
template <class Lut, class Mx>
G2048_HD uint64_t board_move_lean(uint64_t b, uint32_t a, const Lut& lut, const Mx& mx, MoveSummary& s,
                                  uint64_t& nzg) {
    const uint64_t mvert = 0ull - (uint64_t)((a == 0u) | (a == 2u));
    const uint64_t mrev = 0ull - (uint64_t)((a == 1u) | (a == 2u));
    uint64_t f = b ^ ((b ^ transpose(b)) & mvert);
    f ^= (f ^ reverse_rows(f)) & mrev;
    uint32_t o[4], nw[4], fm[4];
#pragma unroll
    for (int j = 0; j < 4; j++) o[j] = (uint32_t)(f >> (16 * j)) & 0xFFFFu;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        nw[j] = (uint32_t)lut(o[j]);
        fm[j] = (uint32_t)mx(o[j]);
    }
    uint64_t g = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) g |= (uint64_t)nw[j] << (16 * j);
    const uint32_t m01 = fm[0] > fm[1] ? fm[0] : fm[1], m23 = fm[2] > fm[3] ? fm[2] : fm[3];
    const uint32_t mf = m01 > m23 ? m01 : m23;
    g ^= (g ^ reverse_rows(g)) & mrev;
    g ^= (g ^ transpose(g)) & mvert;
    nzg = nz_bits(g);
    s.max_e = mf ? mf + 1u : 0u;
    s.overflow = mf == 15u;
    s.count = (uint32_t)(popc64(nz_bits(b)) - popc64(nzg));
    s.sum_e = nib_sum64(b) - nib_sum64(g) + 2u * s.count;
    if (s.overflow) {  // a saturated 15+15 merge: the aggregate is off by one per such merge; sum the lines
        uint32_t se = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const LineMerges m = line_merges(o[j], nw[j]);
            se += m.e0 + m.e1;
        }
        s.sum_e = se;
    }
    s.score = 0u;
    s.list = 0u;
    return g;
}

// nz / equal-neighbour masks of a board, shared by is_done and action_mask
struct BoardBits {
    uint64_t nz, z, eqh, eqv;
};

// the masks with the board's nz_bits already known
G2048_HD BoardBits board_bits_nz(uint64_t b, uint64_t nz) {
    BoardBits r;
    r.nz = nz;
    r.z = ~r.nz & kNibLsb;
    r.eqh = ~nz_bits(b ^ (b >> 4)) & r.nz & kHMask;
    r.eqv = ~nz_bits(b ^ (b >> 16)) & r.nz & kVMask;
    return r;
}

G2048_HD BoardBits board_bits(uint64_t b) { return board_bits_nz(b, nz_bits(b)); }

G2048_HD bool bits_done(const BoardBits& r) { return r.z == 0 && (r.eqh | r.eqv) == 0; }

G2048_HD uint32_t bits_mask(const BoardBits& r) {
    uint32_t up = ((r.z & (r.nz >> 16) & kVMask) | r.eqv) != 0;
    uint32_t down = ((r.nz & (r.z >> 16) & kVMask) | r.eqv) != 0;
    uint32_t left = ((r.z & (r.nz >> 4) & kHMask) | r.eqh) != 0;
    uint32_t right = ((r.nz & (r.z >> 4) & kHMask) | r.eqh) != 0;
    return up | (right << 1) | (down << 2) | (left << 3);
}

// index (0-based) of the k-th empty cell in row-major order (np.argwhere(board == 0)[k], src/game2048.py:109)
G2048_HD uint32_t kth_empty_cell(uint64_t zbits, uint32_t k) {
    uint32_t pos = 0;
    uint32_t c = (uint32_t)popc64(zbits & 0xFFFFFFFFull);
    if (k >= c) { k -= c; zbits >>= 32; pos += 32; }
    c = (uint32_t)popc64(zbits & 0xFFFFull);
    if (k >= c) { k -= c; zbits >>= 16; pos += 16; }
    c = (uint32_t)popc64(zbits & 0xFFull);
    if (k >= c) { k -= c; zbits >>= 8; pos += 8; }
    c = (uint32_t)popc64(zbits & 0xFull);
    if (k >= c) { pos += 4; }
    return pos >> 2;
}

// ---------------------------------------------------------------------------------------------------------
// numpy PCG64 (np.random.default_rng) -- the RNG of Game2048._spawn (src/game2048.py:113,117) and of
// ReinforceAgent.select_action (src/reinforce_agent.py:187).  Restated from numpy's published algorithm.
// ---------------------------------------------------------------------------------------------------------
struct Pcg64 {
    uint64_t s_lo, s_hi, i_lo, i_hi;
    uint32_t has_uint32, uinteger;
};

constexpr uint64_t kPcgMulHi = 0x2360ED051FC65DA4ull;
constexpr uint64_t kPcgMulLo = 0x4385DF649FCCF645ull;

G2048_HD uint64_t mulhi64(uint64_t a, uint64_t b) { return (uint64_t)(((unsigned __int128)a * b) >> 64); }

G2048_HD void pcg_step(Pcg64& g) {
    uint64_t lo = g.s_lo * kPcgMulLo;
    uint64_t hi = mulhi64(g.s_lo, kPcgMulLo) + g.s_lo * kPcgMulHi + g.s_hi * kPcgMulLo;
    uint64_t nlo = lo + g.i_lo;
    g.s_hi = hi + g.i_hi + (nlo < lo);
    g.s_lo = nlo;
}

G2048_HD uint64_t pcg_next64(Pcg64& g) {
    pcg_step(g);
    uint64_t x = g.s_hi ^ g.s_lo;
    uint32_t rot = (uint32_t)(g.s_hi >> 58);
    return (x >> rot) | (x << ((64u - rot) & 63u));
}

G2048_HD uint32_t pcg_next32(Pcg64& g) {
    if (g.has_uint32) {
        g.has_uint32 = 0;
        return g.uinteger;
    }
    uint64_t v = pcg_next64(g);
    g.has_uint32 = 1;
    g.uinteger = (uint32_t)(v >> 32);
    return (uint32_t)v;
}

// Generator.random(): (next_uint64 >> 11) * 2**-53
G2048_HD double pcg_random(Pcg64& g) { return (double)(pcg_next64(g) >> 11) * (1.0 / 9007199254740992.0); }

// Generator.integers(n) for 1 <= n <= 16 (32-bit Lemire with rejection; n == 1 draws nothing)
G2048_HD uint32_t pcg_bounded(Pcg64& g, uint32_t n) {
    if (n <= 1u) return 0u;
    const uint32_t rng = n - 1u;
    uint64_t m = (uint64_t)pcg_next32(g) * n;
    uint32_t left = (uint32_t)m;
    if (left < n) {
        const uint32_t thr = (0xFFFFFFFFu - rng) % n;
        while (left < thr) {
            m = (uint64_t)pcg_next32(g) * n;
            left = (uint32_t)m;
        }
    }
    return (uint32_t)(m >> 32);
}

// SeedSequence(seed).generate_state(4, uint64) -> pcg_setseq_128_srandom_r (np.random.PCG64(seed))
G2048_HD uint32_t ss_hashmix(uint32_t v, uint32_t& hc) {
    v ^= hc;
    hc *= 0x931e8875u;
    v *= hc;
    v ^= v >> 16;
    return v;
}

G2048_HD uint32_t ss_mix(uint32_t x, uint32_t y) {
    uint32_t r = 0xca01f9ddu * x - 0x4973f715u * y;
    return r ^ (r >> 16);
}

G2048_HD Pcg64 pcg_seed(uint64_t seed) {
    const uint32_t w0 = (uint32_t)seed, w1 = (uint32_t)(seed >> 32);
    const bool two = w1 != 0u;  // python int -> uint32 words, little-endian, at least one word
    uint32_t pool[4];
    uint32_t hc = 0x43b0d7e5u;
    pool[0] = ss_hashmix(w0, hc);
    pool[1] = ss_hashmix(two ? w1 : 0u, hc);
    pool[2] = ss_hashmix(0u, hc);
    pool[3] = ss_hashmix(0u, hc);
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
        for (int d = 0; d < 4; d++)
            if (s != d) pool[d] = ss_mix(pool[d], ss_hashmix(pool[s], hc));
    uint32_t w[8];
    uint32_t hb = 0x8b51f9ddu;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint32_t v = pool[i & 3];
        v ^= hb;
        hb *= 0x58f38dedu;
        v *= hb;
        v ^= v >> 16;
        w[i] = v;
    }
    // generate_state(4, uint64) words: v[k] = w[2k] | w[2k+1] << 32; initstate = v0:v1, initseq = v2:v3
    const uint64_t st_hi = ((uint64_t)w[1] << 32) | w[0], st_lo = ((uint64_t)w[3] << 32) | w[2];
    const uint64_t sq_hi = ((uint64_t)w[5] << 32) | w[4], sq_lo = ((uint64_t)w[7] << 32) | w[6];
    Pcg64 g;
    g.i_hi = (sq_hi << 1) | (sq_lo >> 63);
    g.i_lo = (sq_lo << 1) | 1u;
    g.s_lo = 0;
    g.s_hi = 0;
    pcg_step(g);
    uint64_t lo = g.s_lo + st_lo;
    g.s_hi = g.s_hi + st_hi + (lo < g.s_lo);
    g.s_lo = lo;
    pcg_step(g);
    g.has_uint32 = 0;
    g.uinteger = 0;
    return g;
}

// ---------------------------------------------------------------------------------------------------------
// Philox4x32-10 (throughput mode; distributionally equal, not stream-equal, to numpy)
// ---------------------------------------------------------------------------------------------------------
struct U4 {
    uint32_t x, y, z, w;
};

G2048_HD U4 philox4x32(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; r++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
        U4 n;
        n.x = (uint32_t)(p1 >> 32) ^ c.y ^ k0;
        n.y = (uint32_t)p1;
        n.z = (uint32_t)(p0 >> 32) ^ c.w ^ k1;
        n.w = (uint32_t)p0;
        c = n;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// ---------------------------------------------------------------------------------------------------------
// Game2048._spawn (src/game2048.py:108-118): uniform empty cell, then 2 (p=0.9) or 4.
// ---------------------------------------------------------------------------------------------------------
// the spawn with the board's empty-cell bits z (bit 4i = cell i empty) already known; nzbit = the nz_bits bit of
// the new tile (0 if the board was full)
G2048_HD uint64_t spawn_pcg_z(uint64_t b, uint64_t z, Pcg64& g, uint64_t& nzbit) {
    nzbit = 0;
    uint32_t n = (uint32_t)popc64(z);
    if (n == 0u) return b;
    uint32_t k = pcg_bounded(g, n);
    uint32_t cell = kth_empty_cell(z, k);
    uint64_t e = pcg_random(g) < 0.9 ? 1u : 2u;
    nzbit = 1ull << (4u * cell);
    return b | (e << (4u * cell));
}

G2048_HD uint64_t pcg_output(uint64_t s_hi, uint64_t s_lo) {
    const uint64_t x = s_hi ^ s_lo;
    const uint32_t rot = (uint32_t)(s_hi >> 58);
    return (x >> rot) | (x << ((64u - rot) & 63u));
}

// random() < 0.9 on numpy's (next_uint64 >> 11) * 2**-53, as an integer compare: 0.9 (the double) * 2**53 is the
// integer 8106479329266893 (0.9's 52-bit mantissa shifted by 52), and k * 2**-53 < 0.9 <=> k < that integer.
constexpr uint64_t kRandom09 = 8106479329266893ull;

// _spawn (src/game2048.py:108-118) on the numpy PCG64 stream without branches on the common path (the step kernel's
// lean path): the one- and two-step successor states are both formed, and next_uint32's buffer decides which one
// random() draws from -- the same draws as spawn_pcg_z.  A Lemire draw that may be rejected (its low word < n:
// probability < 2^-28) takes the exact path, spawn_pcg_z on the original state.  Requires z != 0 (the board changed,
// so the move emptied at least one cell).
G2048_HD uint64_t spawn_pcg_lean(uint64_t b, uint64_t z, Pcg64& g, uint64_t& nzbit) {
    const uint32_t n = (uint32_t)popc64(z);
    Pcg64 A = g;
    pcg_step(A);
    Pcg64 B = A;
    pcg_step(B);
    const uint64_t oA = pcg_output(A.s_hi, A.s_lo);
    const bool draw = n > 1u;                        // integers(n) draws nothing for n == 1
    const bool fresh = draw && !g.has_uint32;        // next_uint32 takes a new 64-bit output (state -> A)
    const uint32_t u = g.has_uint32 ? g.uinteger : (uint32_t)oA;
    const uint64_t m = (uint64_t)u * n;
    if (draw && (uint32_t)m < n) return spawn_pcg_z(b, z, g, nzbit);   // possible Lemire rejection: exact path
    const uint32_t k = draw ? (uint32_t)(m >> 32) : 0u;
    const uint64_t r_hi = fresh ? B.s_hi : A.s_hi, r_lo = fresh ? B.s_lo : A.s_lo;
    const uint64_t e = (pcg_output(r_hi, r_lo) >> 11) < kRandom09 ? 1u : 2u;
    const uint32_t cell = kth_empty_cell(z, k);
    g.s_hi = r_hi;
    g.s_lo = r_lo;
    g.uinteger = fresh ? (uint32_t)(oA >> 32) : g.uinteger;
    g.has_uint32 = draw ? (g.has_uint32 ^ 1u) : g.has_uint32;
    nzbit = 1ull << (4u * cell);
    return b | (e << (4u * cell));
}

G2048_HD uint64_t spawn_pcg(uint64_t b, Pcg64& g) {
    uint64_t nzbit;
    return spawn_pcg_z(b, ~nz_bits(b) & kNibLsb, g, nzbit);
}

// logits_to_probs (src/MLP.py:139-156) + the action choice of select_action (src/reinforce_agent.py:178-190) for
// one board: where(mask, logits, -1e9), max-shifted softmax in fp32; greedy = argmax of probs*mask (first
// maximum); else Generator.choice(4, p): fp64 cdf normalised by its last entry, searchsorted(side='right') of the
// uniform draw u.  mw: int8[4] mask as one word (byte a = action a); has_mask false = no mask.
G2048_HD uint32_t softmax_select(const float lg[4], uint32_t mw, bool has_mask, bool greedy, double u, float p[4]) {
    const bool m[4] = {(mw & 0xFFu) != 0u, ((mw >> 8) & 0xFFu) != 0u, ((mw >> 16) & 0xFFu) != 0u, (mw >> 24) != 0u};
    float l[4];
    for (int k = 0; k < 4; k++) l[k] = (!has_mask || m[k]) ? lg[k] : -1e9f;
    const float mx = fmaxf(fmaxf(l[0], l[1]), fmaxf(l[2], l[3]));
    float e[4];
    for (int k = 0; k < 4; k++) e[k] = expf(l[k] - mx);
    const float s = ((e[0] + e[1]) + e[2]) + e[3];
    for (int k = 0; k < 4; k++) p[k] = e[k] / s;
    uint32_t act = 0;
    if (greedy) {
        float best = has_mask ? p[0] * (float)m[0] : p[0];
        for (int k = 1; k < 4; k++) {
            const float q = has_mask ? p[k] * (float)m[k] : p[k];
            if (q > best) {
                best = q;
                act = (uint32_t)k;
            }
        }
    } else {
        double cdf[4], acc = 0.0;
        for (int k = 0; k < 4; k++) {
            acc += (double)p[k];
            cdf[k] = acc;
        }
        for (int k = 0; k < 4; k++) act += (cdf[k] / cdf[3] <= u) ? 1u : 0u;
    }
    return act;
}

// Philox spawn: r.x picks the cell (Lemire, no rejection), r.y < 0.9 * 2**32 picks the 2
G2048_HD uint64_t spawn_philox_z(uint64_t b, uint64_t z, U4 r, uint64_t& nzbit) {
    nzbit = 0;
    uint32_t n = (uint32_t)popc64(z);
    if (n == 0u) return b;
    uint32_t k = (uint32_t)(((uint64_t)r.x * n) >> 32);
    uint32_t cell = kth_empty_cell(z, k);
    uint64_t e = r.y < 3865470566u ? 1u : 2u;
    nzbit = 1ull << (4u * cell);
    return b | (e << (4u * cell));
}

G2048_HD uint64_t spawn_philox(uint64_t b, U4 r) {
    uint64_t nzbit;
    return spawn_philox_z(b, ~nz_bits(b) & kNibLsb, r, nzbit);
}

// ---------------------------------------------------------------------------------------------------------
// Game2048Env._compute_reward (src/env.py:197-261), fp64 with the reference's operation order.
// max_tile_e is log2(Game2048Env.max_tile_seen) and is updated in place.
// ---------------------------------------------------------------------------------------------------------
struct RewardCfg {
    int32_t reward_mode, bonus_mode, use_action_mask;
    uint32_t terms;   // reward_terms(*this): set by whoever fills the fields
    double base_reward_scale, empty_tile_reward, merge_reward, bonus_scale, step_reward, endgame_penalty,
        invalid_action_penalty;
};

// The config's branch conditions as one integer word (bits kRw*).  env_reward tests these bits rather than the
// fields: in the step kernel's loop the fp64 `!= 0.0` tests are VALU compares whose loop-invariant 64-bit results
// the compiler hoists and spills to VGPR lanes (a v_readlane each per use); a bit test is one scalar instruction.
constexpr uint32_t kRwInvalidPenalty = 1u, kRwLog2 = 2u, kRwEmpty = 4u, kRwMerge = 8u, kRwEndgame = 16u,
                   kRwBonusRaw = 32u, kRwBonusLog2 = 64u;
G2048_HD uint32_t reward_terms(const RewardCfg& c) {
    return (c.use_action_mask ? 0u : kRwInvalidPenalty) | (c.reward_mode == 0 ? 0u : kRwLog2) |
           (c.empty_tile_reward != 0.0 ? kRwEmpty : 0u) | (c.merge_reward != 0.0 ? kRwMerge : 0u) |
           (c.endgame_penalty != 0.0 ? kRwEndgame : 0u) | (c.bonus_mode == 1 ? kRwBonusRaw : 0u) |
           (c.bonus_mode == 2 ? kRwBonusLog2 : 0u);
}

// final_nz = nz_bits(final board) (the empty-tile term); LOG2_ONLY: the caller guarantees reward_mode "log2" (the
// summary's score is then not read, and need not have been computed).
template <bool LOG2_ONLY = false>
G2048_HD double env_reward_nz(const RewardCfg& c, const MoveSummary& s, uint64_t final_nz, bool done, bool invalid,
                              uint32_t& max_tile_e) {
    uint32_t t = c.terms;
#ifdef __HIP_DEVICE_COMPILE__
    // opaque per call: otherwise each bit test is hoisted out of the caller's loop as a 64-bit lane mask (it guards
    // divergent code) and spilled like the fp64 compares were
    asm volatile("" : "+s"(t));
#endif
    if ((t & kRwInvalidPenalty) && invalid) return c.invalid_action_penalty;
    double r = (LOG2_ONLY || (t & kRwLog2)) ? (double)s.sum_e : (double)s.score;
    r *= c.base_reward_scale;
    if (t & kRwEmpty) {
        const int ne = 16 - popc64(final_nz);
        r += c.empty_tile_reward * (double)ne;
    }
    if (t & kRwMerge) r += c.merge_reward * (double)s.count;
    if (s.max_e >= 3u && s.max_e > max_tile_e) {
        double bonus = 0.0;
        if (t & kRwBonusRaw) bonus = (double)(1u << s.max_e);
        else if (t & kRwBonusLog2) bonus = (double)s.max_e;
        max_tile_e = s.max_e;
        bonus *= c.bonus_scale;
        r += bonus;
    }
    r += c.step_reward;
    if (done && (t & kRwEndgame)) r += c.endgame_penalty;
    return r;
}

G2048_HD double env_reward(const RewardCfg& c, const MoveSummary& s, uint64_t final_board, bool done, bool invalid,
                           uint32_t& max_tile_e) {
    return env_reward_nz<false>(c, s, nz_bits(final_board), done, invalid, max_tile_e);
}

// Flag bits of a step (the G2048_F_* of include/g2048.h; g2048.hip static_asserts they agree).
constexpr uint32_t kFChanged = 1u, kFTerminated = 2u, kFTruncated = 4u, kFInvalid = 8u, kFOverflow = 16u;

// One Game2048Env.step (src/env.py:264-302) on a lane held in values, PCG64 parity stream: move, score, spawn
// only if the board changed (src/game2048.py:40-70), done of the final board, reward (fp64, stored fp32 by the
// caller), truncation at max_steps (< 0 = None).  Updates step_count / max_tile_e / g; returns the new board.
struct StepValues {
    uint64_t board;
    double reward;
    uint32_t flags, score_add;
};

template <class Lut, class Code>
G2048_HD StepValues env_step_pcg(uint64_t b, uint32_t a, uint32_t& step_count, uint32_t& max_tile_e, Pcg64& g,
                                 const RewardCfg& rc, int64_t max_steps, const Lut& lut, const Code& code) {
    const uint32_t sc = step_count + 1u;
    MoveSummary s;
    uint64_t m = board_move_coded<false>(b, a, lut, code, s);
    const bool changed = m != b;
    if (changed) m = spawn_pcg(m, g);
    const BoardBits bits = board_bits(m);
    const bool done = bits_done(bits);
    const bool invalid = !changed && !done;
    StepValues o;
    o.reward = env_reward(rc, s, m, done, invalid, max_tile_e);
    const bool trunc = max_steps >= 0 && (int64_t)sc >= max_steps && !done;
    o.flags = (changed ? kFChanged : 0u) | (done ? kFTerminated : 0u) | (trunc ? kFTruncated : 0u) |
              (invalid ? kFInvalid : 0u) | (s.overflow ? kFOverflow : 0u);
    o.board = m;
    o.score_add = s.score;
    step_count = sc;
    return o;
}

// Dihedral symmetry k of a board (Game2048Env.get_symmetries order, src/env.py:355-396):
// k = 0..3: k counter-clockwise quarter turns (np.rot90 k=1 per step); k = 4..7: fliplr, then (k-4) turns.
G2048_HD uint64_t rot_ccw(uint64_t b) { return transpose(reverse_rows(b)); }  // out[i][j] = b[j][3-i]

G2048_HD uint64_t symmetry_board(uint64_t b, int k) {
    uint64_t x = k >= 4 ? reverse_rows(b) : b;
    const int t = k & 3;
    for (int i = 0; i < t; i++) x = rot_ccw(x);
    return x;
}

// action remap of the same symmetry: rotate_action_ccw90 (a-1)%4, flip_action_horiz 1<->3
G2048_HD uint32_t symmetry_action(uint32_t a, int k) {
    if (k >= 4) a = (a == 1u) ? 3u : (a == 3u ? 1u : a);
    return (a + 4u - (uint32_t)(k & 3)) & 3u;
}

}  // namespace g2048

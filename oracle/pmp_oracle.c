/*
 * oracle/pmp_oracle.c -- CPU restatement of the reference's hot-path algorithms.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker (or the timed CPU
 * baseline).  The product path (python_motion_planning_amd/) never links or calls it.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * src/python_motion_planning/ of Slenderman00/python_motion_planning @ 2025-09-26).
 * Parity of this restatement is pinned by golden vectors generated from the reference
 * itself (tests/golden/make_golden.py) and by the reference's own published
 * 3d_pathfinding_results.csv rows (tests/golden/astar3d_csv.json).
 *
 * Build: oracle/Makefile  (gcc -O2 -ffp-contract=off -fopenmp, no FMA contraction, so
 * every floating-point operation rounds exactly where CPython/numpy round it).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

/* ------------------------------------------------------------------------------------ */
/* CPython 3.10 math.hypot (Modules/mathmodule.c vector_norm), called by                */
/* utils/planner/planner.py:22-23 (Planner.dist), graph_search.py:44 (h), and           */
/* local_planner.py:94-95.  Restated from the published algorithm: scale by a power of  */
/* two, Dekker-split each coordinate, compensated sum of squares, one Newton correction. */
/* ------------------------------------------------------------------------------------ */
static double vnorm2(double a, double b)
{
    const double T27 = 134217729.0; /* 2**27 + 1 */
    double v[2], mx = 0.0;
    int found_nan = 0;
    v[0] = fabs(a);
    v[1] = fabs(b);
    for (int i = 0; i < 2; i++) {
        found_nan |= isnan(v[i]);
        if (v[i] > mx) mx = v[i];
    }
    if (isinf(mx)) return mx;
    if (found_nan) return NAN;
    if (mx == 0.0) return mx;
    int e;
    frexp(mx, &e);
    double csum = 1.0, frac = 0.0, oldcsum, x, t, hi, lo, h;
    if (e >= -1023) {
        double scale = ldexp(1.0, -e);
        for (int i = 0; i < 2; i++) {
            x = v[i] * scale;
            t = x * T27;
            hi = t - (t - x);
            lo = x - hi;
            x = hi * hi;
            oldcsum = csum; csum += x; frac += (oldcsum - csum) + x;
            x = 2.0 * hi * lo;
            oldcsum = csum; csum += x; frac += (oldcsum - csum) + x;
            x = lo * lo;
            oldcsum = csum; csum += x; frac += (oldcsum - csum) + x;
        }
        h = sqrt(csum - 1.0 + frac);
        x = h;
        t = x * T27;
        hi = t - (t - x);
        lo = x - hi;
        x = -hi * hi;
        oldcsum = csum; csum += x; frac += (oldcsum - csum) + x;
        x = -2.0 * hi * lo;
        oldcsum = csum; csum += x; frac += (oldcsum - csum) + x;
        x = -lo * lo;
        oldcsum = csum; csum += x; frac += (oldcsum - csum) + x;
        x = csum - 1.0 + frac;
        return (h + x / (2.0 * h)) / scale;
    }
    for (int i = 0; i < 2; i++) {
        x = v[i] / mx;
        x = x * x;
        oldcsum = csum; csum += x; frac += (oldcsum - csum) + x;
    }
    return mx * sqrt(csum - 1.0 + frac);
}

double oracle_hypot(double a, double b) { return vnorm2(a, b); }

void oracle_hypot_many(const double* a, const double* b, double* out, int64_t n)
{
    for (int64_t i = 0; i < n; i++) out[i] = vnorm2(a[i], b[i]);
}

/* ------------------------------------------------------------------------------------ */
/* CPython heapq (Lib/heapq.py: heappush/_siftdown, heappop/_siftup) used at             */
/* global_planner/graph_search/a_star.py:50,54,76,80, ordered by Node.__lt__             */
/* (utils/environment/node.py:51-54): f = g+h, ties broken by h, nothing else.           */
/* ------------------------------------------------------------------------------------ */
typedef struct {
    double g, h;
    int32_t cell, parent;
} anode_t;

static inline int anode_lt(const anode_t* a, const anode_t* b)
{
    double fa = a->g + a->h, fb = b->g + b->h;
    return fa < fb || (fa == fb && a->h < b->h);
}

static void a_siftdown(anode_t* heap, int64_t startpos, int64_t pos)
{
    anode_t newitem = heap[pos];
    while (pos > startpos) {
        int64_t parentpos = (pos - 1) >> 1;
        if (anode_lt(&newitem, &heap[parentpos])) {
            heap[pos] = heap[parentpos];
            pos = parentpos;
            continue;
        }
        break;
    }
    heap[pos] = newitem;
}

static void a_siftup(anode_t* heap, int64_t endpos, int64_t pos)
{
    int64_t startpos = pos;
    anode_t newitem = heap[pos];
    int64_t childpos = 2 * pos + 1;
    while (childpos < endpos) {
        int64_t rightpos = childpos + 1;
        if (rightpos < endpos && !anode_lt(&heap[childpos], &heap[rightpos])) childpos = rightpos;
        heap[pos] = heap[childpos];
        pos = childpos;
        childpos = 2 * pos + 1;
    }
    heap[pos] = newitem;
    a_siftdown(heap, startpos, pos);
}

/* 8 motions of Grid (utils/environment/env.py:52-55), in this order. */
static const int MX8[8] = {-1, -1, 0, 1, 1, 1, 0, -1};
static const int MY8[8] = {0, 1, 1, 1, 0, -1, -1, -1};

static inline int occ2(const uint8_t* occ, int W, int H, int x, int y)
{
    if (x < 0 || y < 0 || x >= W || y >= H) return 1; /* outside the grid: blocked */
    return occ[(int64_t)x * H + y] != 0;
}

/* GraphSearcher.isCollision, graph_search.py:61-87: endpoints, then both corner cells of a
 * diagonal move (the min/max construction at :78-86 names exactly the two corners). */
static inline int collide2(const uint8_t* occ, int W, int H, int x1, int y1, int x2, int y2)
{
    if (occ2(occ, W, H, x1, y1) || occ2(occ, W, H, x2, y2)) return 1;
    if (x1 != x2 && y1 != y2) {
        if (occ2(occ, W, H, x1, y2) || occ2(occ, W, H, x2, y1)) return 1;
    }
    return 0;
}

/* Return codes for every planner: 0 found, 1 no path, 2 path_cap overflow,
 * 3 heap/expand capacity overflow, 4 reference raises. */

/*
 * AStar.plan  (global_planner/graph_search/a_star.py:39-83) + getNeighbor (:85-96)
 *             + extractPath (:98-117).
 * heuristic: 0 = euclidean (math.hypot), 1 = manhattan (graph_search.py:41-44).
 * path: goal -> start order (reference does not reverse it), cell ids x*H+y.
 * expand (nullable): closure order of CLOSED (list(CLOSED.values()), :64).
 */
int oracle_astar2d(const uint8_t* occ, int W, int H, int heuristic, int sx, int sy, int gx, int gy,
                   double* cost_out, int32_t* path, int path_cap, int32_t* path_len,
                   int32_t* expand, int expand_cap, int32_t* n_expanded, int64_t* counters)
{
    const int64_t ncell = (int64_t)W * H;
    uint8_t* closed = (uint8_t*)calloc((size_t)ncell, 1);
    int32_t* cparent = (int32_t*)malloc(sizeof(int32_t) * (size_t)ncell);
    int64_t cap = 1024, n = 0, npush = 0, npop = 0, nexp = 0, maxn = 1;
    anode_t* heap = (anode_t*)malloc(sizeof(anode_t) * (size_t)cap);
    const double SQ2 = sqrt(2.0);
    int status = 1;
    *path_len = 0;
    *cost_out = 0.0;
    if (!closed || !cparent || !heap) { free(closed); free(cparent); free(heap); return 3; }
    const int32_t start = sx * H + sy, goal = gx * H + gy;
    /* start node: Node(start, start, 0, 0)  (planner.py:15) */
    heap[n++] = (anode_t){0.0, 0.0, start, start};
    npush++;
    while (n > 0) {
        anode_t node;
        n--;
        npop++;
        if (n > 0) {
            node = heap[0];
            heap[0] = heap[n];
            a_siftup(heap, n, 0);
        } else {
            node = heap[0];
        }
        if (closed[node.cell]) continue;
        int x = node.cell / H, y = node.cell % H;
        if (node.cell == goal) {
            closed[node.cell] = 1;
            cparent[node.cell] = node.parent;
            if (expand && nexp < expand_cap) expand[nexp] = node.cell;
            nexp++;
            /* extractPath: walk parents goal -> start, cost += hypot in that order */
            double cost = 0.0;
            int32_t c = goal;
            int32_t len = 0;
            status = 0;
            if (len < path_cap) path[len] = c; else status = 2;
            len++;
            while (c != start) {
                int32_t p = cparent[c];
                cost += vnorm2((double)(p / H - c / H), (double)(p % H - c % H));
                c = p;
                if (len < path_cap) path[len] = c; else status = 2;
                len++;
            }
            *path_len = len;
            *cost_out = cost;
            break;
        }
        for (int m = 0; m < 8; m++) {
            int nx = x + MX8[m], ny = y + MY8[m];
            if (collide2(occ, W, H, x, y, nx, ny)) continue;
            int32_t nc = nx * H + ny;
            if (closed[nc]) continue;
            anode_t nb;
            nb.cell = nc;
            nb.parent = node.cell;
            nb.g = node.g + ((m & 1) ? SQ2 : 1.0);
            if (heuristic == 1)
                nb.h = (double)(abs(gx - nx) + abs(gy - ny));
            else
                nb.h = vnorm2((double)(gx - nx), (double)(gy - ny));
            if (n == cap) {
                cap *= 2;
                anode_t* nh = (anode_t*)realloc(heap, sizeof(anode_t) * (size_t)cap);
                if (!nh) { status = 3; goto done; }
                heap = nh;
            }
            heap[n++] = nb;
            npush++;
            if (n > maxn) maxn = n;
            a_siftdown(heap, 0, n - 1);
            if (nc == goal) break;
        }
        closed[node.cell] = 1;
        cparent[node.cell] = node.parent;
        if (expand && nexp < expand_cap) expand[nexp] = node.cell;
        nexp++;
    }
done:
    *n_expanded = (int32_t)nexp;
    if (counters) { counters[0] = npush; counters[1] = npop; counters[2] = nexp; counters[3] = maxn; }
    if (status == 1) *path_len = 0;
    if (status == 0 && expand && nexp > expand_cap) status = 3;
    free(closed); free(cparent); free(heap);
    return status;
}

/* ------------------------------------------------------------------------------------ */
/* AStar3D.plan (global_planner/graph_search/a_star3d.py:33-78): heap of tuples           */
/* (f, h, counter, node) -> total order; reopening allowed; CLOSED written before the     */
/* goal test; path reversed to start -> goal (:105).                                      */
/* ------------------------------------------------------------------------------------ */
typedef struct {
    double f, h, g;
    int64_t seq;
    int32_t cell, parent;
} a3node_t;

static inline int a3_lt(const a3node_t* a, const a3node_t* b)
{
    if (a->f < b->f) return 1;
    if (a->f > b->f) return 0;
    if (a->h < b->h) return 1;
    if (a->h > b->h) return 0;
    return a->seq < b->seq;
}

static void a3_siftdown(a3node_t* heap, int64_t startpos, int64_t pos)
{
    a3node_t newitem = heap[pos];
    while (pos > startpos) {
        int64_t parentpos = (pos - 1) >> 1;
        if (a3_lt(&newitem, &heap[parentpos])) {
            heap[pos] = heap[parentpos];
            pos = parentpos;
            continue;
        }
        break;
    }
    heap[pos] = newitem;
}

static void a3_siftup(a3node_t* heap, int64_t endpos, int64_t pos)
{
    int64_t startpos = pos;
    a3node_t newitem = heap[pos];
    int64_t childpos = 2 * pos + 1;
    while (childpos < endpos) {
        int64_t rightpos = childpos + 1;
        if (rightpos < endpos && !a3_lt(&heap[childpos], &heap[rightpos])) childpos = rightpos;
        heap[pos] = heap[childpos];
        pos = childpos;
        childpos = 2 * pos + 1;
    }
    heap[pos] = newitem;
    a3_siftdown(heap, startpos, pos);
}

/* 26 motions of Grid3D (utils/environment/env3d.py:56-70), in this order. */
static const int M3[26][3] = {
    {-1, 0, 0}, {-1, 1, 0}, {0, 1, 0}, {1, 1, 0}, {1, 0, 0}, {1, -1, 0}, {0, -1, 0}, {-1, -1, 0},
    {0, 0, 1}, {0, 0, -1},
    {-1, 0, 1}, {-1, 1, 1}, {0, 1, 1}, {1, 1, 1}, {1, 0, 1}, {1, -1, 1}, {0, -1, 1}, {-1, -1, 1},
    {-1, 0, -1}, {-1, 1, -1}, {0, 1, -1}, {1, 1, -1}, {1, 0, -1}, {1, -1, -1}, {0, -1, -1}, {-1, -1, -1}};

static inline int occ3(const uint8_t* occ, int X, int Y, int Z, int x, int y, int z)
{
    if (x < 0 || y < 0 || z < 0 || x >= X || y >= Y || z >= Z) return 1;
    return occ[((int64_t)x * Y + y) * Z + z] != 0;
}

/* GraphSearcher3D.isCollision (graph_search_3d.py:66-107) for unit motions. */
static inline int collide3(const uint8_t* occ, int X, int Y, int Z, int x1, int y1, int z1, int dx, int dy, int dz)
{
    if (occ3(occ, X, Y, Z, x1, y1, z1) || occ3(occ, X, Y, Z, x1 + dx, y1 + dy, z1 + dz)) return 1;
    int changes = (dx != 0) + (dy != 0) + (dz != 0);
    if (changes <= 1) return 0;
    if (changes == 2) {
        if (dx != 0 && dy != 0)
            return occ3(occ, X, Y, Z, x1 + dx, y1, z1) || occ3(occ, X, Y, Z, x1, y1 + dy, z1);
        if (dx != 0 && dz != 0)
            return occ3(occ, X, Y, Z, x1 + dx, y1, z1) || occ3(occ, X, Y, Z, x1, y1, z1 + dz);
        return occ3(occ, X, Y, Z, x1, y1 + dy, z1) || occ3(occ, X, Y, Z, x1, y1, z1 + dz);
    }
    return occ3(occ, X, Y, Z, x1 + dx, y1, z1) || occ3(occ, X, Y, Z, x1, y1 + dy, z1) ||
           occ3(occ, X, Y, Z, x1, y1, z1 + dz);
}

/* heuristic: 0 euclidean = math.sqrt(dx**2+dy**2+dz**2) (graph_search_3d.py:40-50), 1 manhattan.
 * path: start -> goal.  expand: distinct CLOSED keys in first-insertion order.
 * Unreachable -> status 1 with cost = inf (a_star3d.py:77-78). */
int oracle_astar3d(const uint8_t* occ, int X, int Y, int Z, int heuristic, const int32_t* s, const int32_t* g,
                   double* cost_out, int32_t* path, int path_cap, int32_t* path_len,
                   int32_t* expand, int expand_cap, int32_t* n_expanded, int64_t* counters)
{
    const int64_t ncell = (int64_t)X * Y * Z;
    double* cg = (double*)malloc(sizeof(double) * (size_t)ncell);
    int32_t* cparent = (int32_t*)malloc(sizeof(int32_t) * (size_t)ncell);
    uint8_t* closed = (uint8_t*)calloc((size_t)ncell, 1);
    int64_t cap = 1024, n = 0, npush = 0, npop = 0, nexp = 0, seq = 0, nclose = 0;
    a3node_t* heap = (a3node_t*)malloc(sizeof(a3node_t) * (size_t)cap);
    int status = 1;
    *path_len = 0;
    *cost_out = INFINITY;
    if (!cg || !cparent || !closed || !heap) { free(cg); free(cparent); free(closed); free(heap); return 3; }
    const int gx = g[0], gy = g[1], gz = g[2];
    const int32_t start = (s[0] * Y + s[1]) * Z + s[2], goal = (gx * Y + gy) * Z + gz;
#define H3(x, y, z)                                                                                     \
    (heuristic == 1 ? (double)(abs(gx - (x)) + abs(gy - (y)) + abs(gz - (z)))                         \
                    : sqrt((double)((gx - (x)) * (gx - (x)) + (gy - (y)) * (gy - (y)) + (gz - (z)) * (gz - (z)))))
    {
        double h0 = H3(s[0], s[1], s[2]);
        heap[n++] = (a3node_t){0.0 + h0, h0, 0.0, seq++, start, start};
        npush++;
    }
    while (n > 0) {
        a3node_t node;
        n--;
        npop++;
        if (n > 0) {
            node = heap[0];
            heap[0] = heap[n];
            a3_siftup(heap, n, 0);
        } else {
            node = heap[0];
        }
        if (closed[node.cell] && node.g >= cg[node.cell]) continue;
        if (!closed[node.cell]) {
            if (expand && nclose < expand_cap) expand[nclose] = node.cell;
            nclose++;
        }
        closed[node.cell] = 1;
        cg[node.cell] = node.g;
        cparent[node.cell] = node.parent;
        nexp++;
        int z = node.cell % Z, y = (node.cell / Z) % Y, x = node.cell / (Y * Z);
        if (node.cell == goal) {
            /* extractPath (:86-106): cost += dist(node, parent) goal -> start, then reverse */
            double cost = 0.0;
            int32_t c = goal;
            int32_t len = 1;
            while (c != start) {
                int32_t p = cparent[c];
                int ddx = p / (Y * Z) - c / (Y * Z), ddy = (p / Z) % Y - (c / Z) % Y, ddz = p % Z - c % Z;
                cost += sqrt((double)(ddx * ddx + ddy * ddy + ddz * ddz));
                c = p;
                len++;
            }
            status = 0;
            if (len > path_cap) status = 2;
            else {
                c = goal;
                int32_t i = len - 1;
                path[i--] = c;
                while (c != start) { c = cparent[c]; path[i--] = c; }
            }
            *path_len = len;
            *cost_out = cost;
            break;
        }
        for (int m = 0; m < 26; m++) {
            int dx = M3[m][0], dy = M3[m][1], dz = M3[m][2];
            if (collide3(occ, X, Y, Z, x, y, z, dx, dy, dz)) continue;
            int nx = x + dx, ny = y + dy, nz = z + dz;
            int32_t nc = (nx * Y + ny) * Z + nz;
            double tg = node.g + sqrt((double)(dx * dx + dy * dy + dz * dz));
            if (closed[nc] && tg >= cg[nc]) continue;
            double hn = H3(nx, ny, nz);
            if (n == cap) {
                cap *= 2;
                a3node_t* nh = (a3node_t*)realloc(heap, sizeof(a3node_t) * (size_t)cap);
                if (!nh) { status = 3; goto done3; }
                heap = nh;
            }
            heap[n++] = (a3node_t){tg + hn, hn, tg, seq++, nc, node.cell};
            npush++;
            a3_siftdown(heap, 0, n - 1);
        }
    }
#undef H3
done3:
    *n_expanded = (int32_t)nclose;
    if (counters) { counters[0] = npush; counters[1] = npop; counters[2] = nexp; }
    if (status == 1) { *path_len = 0; *cost_out = INFINITY; }
    if (status == 0 && expand && nclose > expand_cap) status = 3;
    free(cg); free(cparent); free(closed); free(heap);
    return status;
}

/* ------------------------------------------------------------------------------------ */
/* DStar (global_planner/graph_search/d_star.py:37-291): list-semantics OPEN.             */
/*  min_state = first element of minimal k in list order (:220-227)                       */
/*  delete    = list.remove -> first occurrence; sets CLOSED only if OPEN (:250-259)      */
/*  insert    = append always, k rule by tag (:236-248)                                    */
/* ------------------------------------------------------------------------------------ */
enum { T_NEW = 0, T_OPEN = 1, T_CLOSED = 2 };

typedef struct {
    double* h;
    double* k;
    int32_t* parent; /* -1 = None */
    uint8_t* t;
    int32_t* open;
    int64_t nopen, capopen;
} dstate_t;

static int d_insert(dstate_t* S, int32_t c, double hnew)
{
    if (S->t[c] == T_NEW) S->k[c] = hnew;
    else if (S->t[c] == T_OPEN) S->k[c] = fmin(S->k[c], hnew);
    else S->k[c] = fmin(S->h[c], hnew);
    S->h[c] = hnew;
    S->t[c] = T_OPEN;
    if (S->nopen == S->capopen) {
        int64_t nc = S->capopen * 2;
        int32_t* no = (int32_t*)realloc(S->open, sizeof(int32_t) * (size_t)nc);
        if (!no) return -1;
        S->open = no;
        S->capopen = nc;
    }
    S->open[S->nopen++] = c;
    return 0;
}

/* python min(key=...) keeps the first minimal element: strict '<' while scanning */
static int64_t d_minpos(const dstate_t* S)
{
    if (S->nopen == 0) return -1;
    int64_t best = 0;
    double bk = S->k[S->open[0]];
    for (int64_t i = 1; i < S->nopen; i++) {
        double kk = S->k[S->open[i]];
        if (kk < bk) { bk = kk; best = i; }
    }
    return best;
}

/* neighbours of cell c that pass isCollision (d_star.py:276-291); returns count */
static int d_neighbors(const uint8_t* occ, int W, int H, int32_t c, int32_t* out, double* cost)
{
    int x = c / H, y = c % H, k = 0;
    const double SQ2 = sqrt(2.0);
    for (int m = 0; m < 8; m++) {
        int nx = x + MX8[m], ny = y + MY8[m];
        if (collide2(occ, W, H, x, y, nx, ny)) continue;
        out[k] = nx * H + ny;
        cost[k] = (m & 1) ? SQ2 : 1.0; /* GraphSearcher.cost -> Planner.dist = hypot(1,1) == sqrt(2) */
        k++;
    }
    return k;
}

/* Returns status; *n_process = number of processState calls (len(EXPAND)).
 * path: start -> goal (d_star.py:136-156). status 4 = reference raises AttributeError
 * (OPEN empties: min_k on None at :234). */
int oracle_dstar2d(const uint8_t* occ, int W, int H, int sx, int sy, int gx, int gy, double* cost_out,
                   int32_t* path, int path_cap, int32_t* path_len, int64_t* n_process, int64_t max_process)
{
    const int64_t ncell = (int64_t)W * H;
    dstate_t S;
    S.h = (double*)malloc(sizeof(double) * (size_t)ncell);
    S.k = (double*)malloc(sizeof(double) * (size_t)ncell);
    S.parent = (int32_t*)malloc(sizeof(int32_t) * (size_t)ncell);
    S.t = (uint8_t*)malloc((size_t)ncell);
    S.capopen = 1024;
    S.nopen = 0;
    S.open = (int32_t*)malloc(sizeof(int32_t) * (size_t)S.capopen);
    int status = 0;
    *path_len = 0;
    *cost_out = 0.0;
    *n_process = 0;
    for (int64_t i = 0; i < ncell; i++) {
        S.h[i] = INFINITY;
        S.k[i] = INFINITY;
        S.parent[i] = -1;
        S.t[i] = T_NEW;
    }
    const int32_t start = sx * H + sy, goal = gx * H + gy;
    S.h[goal] = 0.0; /* DNode(goal, None, 'NEW', 0, inf) (:58) */
    d_insert(&S, goal, 0.0);
    int32_t nb[8];
    double nc[8];
    int64_t np = 0;
    for (;;) {
        /* processState (:158-218) */
        int64_t pos = d_minpos(&S);
        np++;
        if (pos < 0) { status = 4; break; } /* unreachable in practice: OPEN non-empty here */
        int32_t x = S.open[pos];
        double k_old = S.k[x];
        if (S.t[x] == T_OPEN) S.t[x] = T_CLOSED;
        memmove(&S.open[pos], &S.open[pos + 1], sizeof(int32_t) * (size_t)(S.nopen - pos - 1));
        S.nopen--;
        int nn;
        if (k_old < S.h[x]) {
            nn = d_neighbors(occ, W, H, x, nb, nc);
            for (int i = 0; i < nn; i++) {
                int32_t y = nb[i];
                if (S.h[y] <= k_old && S.h[x] > S.h[y] + nc[i]) {
                    S.parent[x] = y;
                    S.h[x] = S.h[y] + nc[i];
                }
            }
        }
        nn = d_neighbors(occ, W, H, x, nb, nc);
        if (k_old == S.h[x]) {
            for (int i = 0; i < nn; i++) {
                int32_t y = nb[i];
                if (S.t[y] == T_NEW || (S.parent[y] == x && S.h[y] != S.h[x] + nc[i]) ||
                    (S.parent[y] != x && S.h[y] > S.h[x] + nc[i])) {
                    S.parent[y] = x;
                    if (d_insert(&S, y, S.h[x] + nc[i])) { status = 3; goto ddone; }
                }
            }
        } else {
            for (int i = 0; i < nn; i++) {
                int32_t y = nb[i];
                if (S.t[y] == T_NEW || (S.parent[y] == x && S.h[y] != S.h[x] + nc[i])) {
                    S.parent[y] = x;
                    if (d_insert(&S, y, S.h[x] + nc[i])) { status = 3; goto ddone; }
                } else if (S.parent[y] != x && S.h[y] > S.h[x] + nc[i]) {
                    if (d_insert(&S, x, S.h[x])) { status = 3; goto ddone; }
                } else if (S.parent[y] != x && S.h[x] > S.h[y] + nc[i] && S.t[y] == T_CLOSED && S.h[y] > k_old) {
                    if (d_insert(&S, y, S.h[y])) { status = 3; goto ddone; }
                }
            }
        }
        if (S.nopen == 0) { status = 4; break; } /* return self.min_k -> None.k raises */
        if (S.t[start] == T_CLOSED) break;
        if (max_process > 0 && np >= max_process) { status = 3; break; }
    }
    if (status == 0) {
        double cost = 0.0;
        int32_t c = start;
        int32_t len = 0;
        if (len < path_cap) path[len] = c; else status = 2;
        len++;
        while (c != goal) {
            int32_t p = S.parent[c];
            if (p < 0) { status = 4; break; } /* closed_list[None] -> KeyError in reference */
            int cx = c / H, cy = c % H, px = p / H, py = p % H;
            if (collide2(occ, W, H, cx, cy, px, py)) cost += INFINITY;
            else cost += vnorm2((double)(px - cx), (double)(py - cy));
            c = p;
            if (len < path_cap) path[len] = c; else status = 2;
            len++;
            if (len > ncell + 1) { status = 4; break; } /* parent cycle: reference loops forever */
        }
        *path_len = len;
        *cost_out = cost;
    }
ddone:
    *n_process = np;
    free(S.h); free(S.k); free(S.parent); free(S.t); free(S.open);
    return status;
}

/* Batch of 2D A* queries on one grid, OpenMP over queries (the CPU baseline of bench.py).
 * path: [nq][path_cap] goal->start cells; counters [nq][4] (push, pop, expansions, max heap).
 * nthreads <= 0: OpenMP default.  Returns the number of queries with status 0. */
int oracle_astar2d_batch(const uint8_t* occ, int W, int H, int heuristic, const int32_t* starts,
                         const int32_t* goals, int nq, double* cost, int32_t* path, int path_cap,
                         int32_t* path_len, int32_t* n_expanded, int64_t* counters, int32_t* status,
                         int nthreads)
{
    int found = 0;
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) reduction(+ : found)
    for (int q = 0; q < nq; q++) {
        status[q] = oracle_astar2d(occ, W, H, heuristic, starts[2 * q], starts[2 * q + 1], goals[2 * q],
                                   goals[2 * q + 1], &cost[q], path + (int64_t)q * path_cap, path_cap,
                                   &path_len[q], NULL, 0, &n_expanded[q], counters ? counters + 4 * (int64_t)q : NULL);
        found += status[q] == 0;
    }
    return found;
}

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

/* ThetaStar.lineOfSight (global_planner/graph_search/theta_star.py:110-171): Bresenham from
 * (x1, y1) to (x2, y2).  tau = (d_y - d_x) / 2 is a half-integer, so `e > tau` is compared as
 * 2e > (d_y - d_x) in integers.  Cells off the grid are not in the obstacle set (a set lookup), but
 * a line between two in-grid endpoints never leaves the grid's bounding box anyway. */
static int los2(const uint8_t* occ, int W, int H, int x1, int y1, int x2, int y2)
{
    if (occ2(occ, W, H, x1, y1) || occ2(occ, W, H, x2, y2)) return 0; /* also the range checks */
    const int dx = abs(x2 - x1), dy = abs(y2 - y1);
    const int sx = x2 > x1 ? 1 : (x2 < x1 ? -1 : 0), sy = y2 > y1 ? 1 : (y2 < y1 ? -1 : 0);
    int x = x1, y = y1, e = 0;
    if (dx > dy) {
        const int T = dy - dx;
        while (x != x2) {
            if (2 * e > T) { x += sx; e -= dy; }
            else if (2 * e < T) { y += sy; e += dx; }
            else { x += sx; y += sy; e += dx - dy; }
            if (x >= 0 && y >= 0 && x < W && y < H && occ[(int64_t)x * H + y]) return 0;
        }
    } else {
        const int T = dx - dy;
        while (y != y2) {
            if (2 * e > T) { y += sy; e -= dx; }
            else if (2 * e < T) { x += sx; e += dy; }
            else { x += sx; y += sy; e += dy - dx; }
            if (x >= 0 && y >= 0 && x < W && y < H && occ[(int64_t)x * H + y]) return 0;
        }
    }
    return 1;
}

/* Return codes for every planner: 0 found, 1 no path, 2 path_cap overflow,
 * 3 heap/expand capacity overflow, 4 reference raises. */

/*
 * AStar.plan  (global_planner/graph_search/a_star.py:39-83) + getNeighbor (:85-96)
 *             + extractPath (:98-117), and the two planners that share its loop:
 *   algo 0: AStar      node_n.h = h(node_n)                            (a_star.py:71-72)
 *   algo 1: Dijkstra   node_n.h = 0                                    (dijkstra.py:73-74)
 *   algo 2: GBFS       node_n.h = h(node_n), node_n.g = 0              (gbfs.py:73-75)
 *   algo 3: ThetaStar  after path 1, updateVertex(CLOSED[node.parent], node_n): lineOfSight(node_n,
 *                      parent) and parent.g + dist <= node_n.g -> path 2  (theta_star.py:44-108)
 *   algo 4: LazyThetaStar  updateVertex without the line of sight at the push; at the pop, no
 *                      lineOfSight(parent, node) -> g = min over CLOSED neighbours (first minimum in
 *                      motion order), g = inf if none  (lazy_theta_star.py:38-114)
 * (Dijkstra/GBFS also skip neighbours in obstacles, dijkstra.py:66-67 / gbfs.py:66-67: a no-op,
 * getNeighbor never returns one.)  All of them push the start as Node(start, start, 0, 0).
 * Theta*'s parents are any cell; extractPath is AStar's (hypot per hop, goal -> start).
 * heuristic: 0 = euclidean (math.hypot), 1 = manhattan (graph_search.py:41-44).
 * path: goal -> start order (reference does not reverse it), cell ids x*H+y.
 * expand (nullable): closure order of CLOSED (list(CLOSED.values()), :64).
 */
int oracle_graph2d(int algo, const uint8_t* occ, int W, int H, int heuristic, int sx, int sy, int gx, int gy,
                   double* cost_out, int32_t* path, int path_cap, int32_t* path_len,
                   int32_t* expand, int expand_cap, int32_t* n_expanded, int64_t* counters)
{
    const int64_t ncell = (int64_t)W * H;
    uint8_t* closed = (uint8_t*)calloc((size_t)ncell, 1);
    int32_t* cparent = (int32_t*)malloc(sizeof(int32_t) * (size_t)ncell);
    double* cg = algo >= 3 ? (double*)malloc(sizeof(double) * (size_t)ncell) : NULL; /* CLOSED[c].g */
    int64_t cap = 1024, n = 0, npush = 0, npop = 0, nexp = 0, maxn = 1;
    anode_t* heap = (anode_t*)malloc(sizeof(anode_t) * (size_t)cap);
    const double SQ2 = sqrt(2.0);
    int status = 1;
    *path_len = 0;
    *cost_out = 0.0;
    if (!closed || !cparent || !heap || (algo >= 3 && !cg)) { free(closed); free(cparent); free(heap); free(cg); return 3; }
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
        if (algo == 4 && closed[node.parent]) {
            /* set vertex (lazy_theta_star.py:55-65); it runs before the CLOSED check there, but on a
             * node that check then skips it changes nothing */
            const int px = node.parent / H, py = node.parent % H;
            if (!los2(occ, W, H, px, py, x, y)) {
                node.g = INFINITY;
                for (int m = 0; m < 8; m++) {
                    int nx = x + MX8[m], ny = y + MY8[m];
                    if (collide2(occ, W, H, x, y, nx, ny)) continue;
                    int32_t nc = nx * H + ny;
                    if (!closed[nc]) continue;
                    const double c = cg[nc] + ((m & 1) ? SQ2 : 1.0);
                    if (node.g > c) { node.g = c; node.parent = nc; }
                }
            }
        }
        if (node.cell == goal) {
            closed[node.cell] = 1;
            cparent[node.cell] = node.parent;
            if (cg) cg[node.cell] = node.g;
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
            nb.g = algo == 2 ? 0.0 : node.g + ((m & 1) ? SQ2 : 1.0);
            if (algo == 1)
                nb.h = 0.0;
            else if (heuristic == 1)
                nb.h = (double)(abs(gx - nx) + abs(gy - ny));
            else
                nb.h = vnorm2((double)(gx - nx), (double)(gy - ny));
            if (algo >= 3 && closed[node.parent]) { /* updateVertex(CLOSED[node.parent], node_n) */
                const int px = node.parent / H, py = node.parent % H;
                const double g2 = cg[node.parent] + vnorm2((double)(px - nx), (double)(py - ny));
                if (g2 <= nb.g && (algo == 4 || los2(occ, W, H, nx, ny, px, py))) {
                    nb.g = g2;
                    nb.parent = node.parent;
                }
            }
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
        if (cg) cg[node.cell] = node.g;
        if (expand && nexp < expand_cap) expand[nexp] = node.cell;
        nexp++;
    }
done:
    *n_expanded = (int32_t)nexp;
    if (counters) { counters[0] = npush; counters[1] = npop; counters[2] = nexp; counters[3] = maxn; }
    if (status == 1) *path_len = 0;
    if (status == 0 && expand && nexp > expand_cap) status = 3;
    free(closed); free(cparent); free(heap); free(cg);
    return status;
}

int oracle_astar2d(const uint8_t* occ, int W, int H, int heuristic, int sx, int sy, int gx, int gy,
                   double* cost_out, int32_t* path, int path_cap, int32_t* path_len,
                   int32_t* expand, int expand_cap, int32_t* n_expanded, int64_t* counters)
{
    return oracle_graph2d(0, occ, W, H, heuristic, sx, sy, gx, gy, cost_out, path, path_cap, path_len, expand,
                          expand_cap, n_expanded, counters);
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
 * Unreachable -> status 1 with cost = inf (a_star3d.py:77-78).
 * algo 0: AStar3D.  algo 1: Dijkstra3D (dijkstra3d.py:39-87): key (g, 0.0, counter), start h = 0,
 * the same reopening rules; its getNeighbor (:89-126) adds an in-bounds test and face checks that
 * equal isCollision's, so with out-of-grid cells blocked it is this loop with h = 0.
 * algo 2: GBFS3D (gbfs3d.py:34-82): key (h, counter), CLOSED membership tests (:55, :74) -- this
 * loop with every g = 0: (f, h, counter) = (h, h, counter), and `g >= closed g` is always true. */
int oracle_graph3d(int algo, const uint8_t* occ, int X, int Y, int Z, int heuristic, const int32_t* s,
                   const int32_t* g, double* cost_out, int32_t* path, int path_cap, int32_t* path_len,
                   int32_t* expand, int expand_cap, int32_t* n_expanded, int64_t* counters)
{
    const int64_t ncell = (int64_t)X * Y * Z;
    double* cg = (double*)malloc(sizeof(double) * (size_t)ncell);
    int32_t* cparent = (int32_t*)malloc(sizeof(int32_t) * (size_t)ncell);
    uint8_t* closed = (uint8_t*)calloc((size_t)ncell, 1);
    int64_t cap = 1024, n = 0, npush = 0, npop = 0, nexp = 0, seq = 0, nclose = 0, maxn = 1;
    a3node_t* heap = (a3node_t*)malloc(sizeof(a3node_t) * (size_t)cap);
    int status = 1;
    *path_len = 0;
    *cost_out = INFINITY;
    if (!cg || !cparent || !closed || !heap) { free(cg); free(cparent); free(closed); free(heap); return 3; }
    const int gx = g[0], gy = g[1], gz = g[2];
    const int32_t start = (s[0] * Y + s[1]) * Z + s[2], goal = (gx * Y + gy) * Z + gz;
#define H3(x, y, z)                                                                                     \
    (algo == 1 ? 0.0 : heuristic == 1 ? (double)(abs(gx - (x)) + abs(gy - (y)) + abs(gz - (z)))       \
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
            double tg = algo == 2 ? 0.0 : node.g + sqrt((double)(dx * dx + dy * dy + dz * dz));
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
            if (n > maxn) maxn = n;
            a3_siftdown(heap, 0, n - 1);
        }
    }
#undef H3
done3:
    *n_expanded = (int32_t)nclose;
    if (counters) { counters[0] = npush; counters[1] = npop; counters[2] = nexp; counters[3] = maxn; }
    if (status == 1) { *path_len = 0; *cost_out = INFINITY; }
    if (status == 0 && expand && nclose > expand_cap) status = 3;
    free(cg); free(cparent); free(closed); free(heap);
    return status;
}

int oracle_astar3d(const uint8_t* occ, int X, int Y, int Z, int heuristic, const int32_t* s, const int32_t* g,
                   double* cost_out, int32_t* path, int path_cap, int32_t* path_len,
                   int32_t* expand, int expand_cap, int32_t* n_expanded, int64_t* counters)
{
    return oracle_graph3d(0, occ, X, Y, Z, heuristic, s, g, cost_out, path, path_cap, path_len, expand, expand_cap,
                          n_expanded, counters);
}

/* ------------------------------------------------------------------------------------ */
/* ThetaStar3D / LazyThetaStar3D (global_planner/graph_search/theta_star3d.py:38-232,      */
/* lazy_theta_star3d.py:41-252): AStar3D's (f, h, counter) heap and reopening rules, with  */
/* any-voxel parents.                                                                      */
/* ------------------------------------------------------------------------------------ */

/* lineOfSight (theta_star3d.py:139-213 == lazy_theta_star3d.py:158-233): integer Bresenham from a
 * to b along the dominant axis; both endpoints must be free; every voxel after a (b included) must
 * be in the grid and free. */
static int los3(const uint8_t* occ, int X, int Y, int Z, int x0, int y0, int z0, int x1, int y1, int z1)
{
    if (occ3(occ, X, Y, Z, x0, y0, z0) || occ3(occ, X, Y, Z, x1, y1, z1)) return 0;
    const int dx = abs(x1 - x0), dy = abs(y1 - y0), dz = abs(z1 - z0);
    const int sx = x1 >= x0 ? 1 : -1, sy = y1 >= y0 ? 1 : -1, sz = z1 >= z0 ? 1 : -1;
    int x = x0, y = y0, z = z0;
    if (dx >= dy && dx >= dz) {
        int ey = dx / 2, ez = dx / 2;
        while (x != x1) {
            x += sx; ey -= dy; ez -= dz;
            if (ey < 0) { y += sy; ey += dx; }
            if (ez < 0) { z += sz; ez += dx; }
            if (occ3(occ, X, Y, Z, x, y, z)) return 0;
        }
        return 1;
    }
    if (dy >= dx && dy >= dz) {
        int ex = dy / 2, ez = dy / 2;
        while (y != y1) {
            y += sy; ex -= dx; ez -= dz;
            if (ex < 0) { x += sx; ex += dy; }
            if (ez < 0) { z += sz; ez += dy; }
            if (occ3(occ, X, Y, Z, x, y, z)) return 0;
        }
        return 1;
    }
    int ex = dz / 2, ey = dz / 2;
    while (z != z1) {
        z += sz; ex -= dx; ey -= dy;
        if (ex < 0) { x += sx; ex += dz; }
        if (ey < 0) { y += sy; ey += dz; }
        if (occ3(occ, X, Y, Z, x, y, z)) return 0;
    }
    return 1;
}

/* Planner3D.dist (utils/planner/planner3d.py:22-27): math.sqrt of the integer sum of squares */
static inline double dist3c(int64_t YZ, int Z, int32_t a, int32_t b)
{
    const int dx = (int)(a / YZ) - (int)(b / YZ), dy = (int)((a / Z) % (YZ / Z)) - (int)((b / Z) % (YZ / Z)),
              dz = (int)(a % Z) - (int)(b % Z);
    return sqrt((double)(dx * dx + dy * dy + dz * dz));
}

int oracle_theta3d(int lazy, const uint8_t* occ, int X, int Y, int Z, int heuristic, const int32_t* s,
                   const int32_t* g, double* cost_out, int32_t* path, int path_cap, int32_t* path_len,
                   int32_t* expand, int expand_cap, int32_t* n_expanded, int64_t* counters)
{
    const int64_t ncell = (int64_t)X * Y * Z, YZ = (int64_t)Y * Z;
    double* cg = (double*)malloc(sizeof(double) * (size_t)ncell);
    int32_t* cparent = (int32_t*)malloc(sizeof(int32_t) * (size_t)ncell);
    uint8_t* closed = (uint8_t*)calloc((size_t)ncell, 1);
    int64_t cap = 1024, n = 0, npush = 0, npop = 0, nexp = 0, seq = 0, nclose = 0, maxn = 1;
    a3node_t* heap = (a3node_t*)malloc(sizeof(a3node_t) * (size_t)cap);
    int status = 1;
    *path_len = 0;
    *cost_out = INFINITY;
    if (!cg || !cparent || !closed || !heap) { free(cg); free(cparent); free(closed); free(heap); return 3; }
    const int gx = g[0], gy = g[1], gz = g[2];
    const int32_t start = (s[0] * Y + s[1]) * Z + s[2], goal = (gx * Y + gy) * Z + gz;
#define H3T(x, y, z)                                                                                    \
    (heuristic == 1 ? (double)(abs(gx - (x)) + abs(gy - (y)) + abs(gz - (z)))                         \
                    : sqrt((double)((gx - (x)) * (gx - (x)) + (gy - (y)) * (gy - (y)) + (gz - (z)) * (gz - (z)))))
#define CX(c) ((int)((c) / YZ))
#define CY(c) ((int)(((c) / Z) % Y))
#define CZ(c) ((int)((c) % Z))
    {
        double h0 = H3T(s[0], s[1], s[2]);
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
        int z = CZ(node.cell), y = CY(node.cell), x = CX(node.cell);
        if (lazy) {
            /* lazy_theta_star3d.py:60-71: the parent is CLOSED (it expanded this node or its parent) */
            const int32_t p = node.parent;
            if (!los3(occ, X, Y, Z, CX(p), CY(p), CZ(p), x, y, z)) {
                node.g = INFINITY;
                for (int m = 0; m < 26; m++) {
                    int dx = M3[m][0], dy = M3[m][1], dz = M3[m][2];
                    if (collide3(occ, X, Y, Z, x, y, z, dx, dy, dz)) continue;
                    int32_t nc = ((x + dx) * Y + (y + dy)) * Z + (z + dz);
                    if (!closed[nc]) continue;
                    double ng = cg[nc] + sqrt((double)(dx * dx + dy * dy + dz * dz));
                    if (ng < node.g) { node.g = ng; node.parent = nc; }
                }
            }
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
        if (node.cell == goal) {
            double cost = 0.0;
            int32_t c = goal, len = 1;
            while (c != start) {
                int32_t p = cparent[c];
                cost += dist3c(YZ, Z, c, p);
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
        const int32_t np_ = node.parent;  /* node_p = CLOSED.get(node.parent): always present */
        for (int m = 0; m < 26; m++) {
            int dx = M3[m][0], dy = M3[m][1], dz = M3[m][2];
            if (collide3(occ, X, Y, Z, x, y, z, dx, dy, dz)) continue;
            int nx = x + dx, ny = y + dy, nz = z + dz;
            int32_t nc = (nx * Y + ny) * Z + nz;
            double g1 = node.g + sqrt((double)(dx * dx + dy * dy + dz * dz));
            if (closed[nc] && g1 >= cg[nc]) continue;
            double qg = g1;
            int32_t qp = node.cell;
            /* updateVertex (theta_star3d.py:102-110 with lineOfSight(q, node_p); lazy_theta_star3d.py:120-128
             * without it) */
            if (lazy || los3(occ, X, Y, Z, nx, ny, nz, CX(np_), CY(np_), CZ(np_))) {
                double alt = cg[np_] + dist3c(YZ, Z, nc, np_);
                if (alt < qg) { qg = alt; qp = np_; }
            }
            double hn = H3T(nx, ny, nz);
            if (n == cap) {
                cap *= 2;
                a3node_t* nh = (a3node_t*)realloc(heap, sizeof(a3node_t) * (size_t)cap);
                if (!nh) { status = 3; goto donet; }
                heap = nh;
            }
            heap[n++] = (a3node_t){qg + hn, hn, qg, seq++, nc, qp};
            npush++;
            if (n > maxn) maxn = n;
            a3_siftdown(heap, 0, n - 1);
        }
    }
#undef H3T
#undef CX
#undef CY
#undef CZ
donet:
    *n_expanded = (int32_t)nclose;
    if (counters) { counters[0] = npush; counters[1] = npop; counters[2] = nexp; counters[3] = maxn; }
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
    int32_t goal_slot, goal_cell; /* start == goal: the goal object lives in slot W*H (d_star.py:66-68) */
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
int oracle_dstar2d_onpress(const uint8_t* occ_in, int W, int H, int sx, int sy, int gx, int gy, const int32_t* presses,
                           int npress, double* cost, int32_t* path, int path_cap, int32_t* plen, int64_t* nproc,
                           int32_t* status, int64_t max_process);

int oracle_dstar2d(const uint8_t* occ, int W, int H, int sx, int sy, int gx, int gy, double* cost_out,
                   int32_t* path, int path_cap, int32_t* path_len, int64_t* n_process, int64_t max_process)
{
    /* DStar.plan: the OnPress restatement with no presses (one processState loop for both) */
    int32_t st;
    oracle_dstar2d_onpress(occ, W, H, sx, sy, gx, gy, NULL, 0, cost_out, path, path_cap, path_len, n_process, &st,
                           max_process);
    return st;
}

/* Batch of 2D A* queries on one grid, OpenMP over queries (the CPU baseline of bench.py).
 * path: [nq][path_cap] goal->start cells; counters [nq][4] (push, pop, expansions, max heap).
 * nthreads <= 0: OpenMP default.  Returns the number of queries with status 0. */
int oracle_graph2d_batch(int algo, const uint8_t* occ, int W, int H, int heuristic, const int32_t* starts,
                         const int32_t* goals, int nq, double* cost, int32_t* path, int path_cap,
                         int32_t* path_len, int32_t* n_expanded, int64_t* counters, int32_t* status,
                         int nthreads)
{
    int found = 0;
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) reduction(+ : found)
    for (int q = 0; q < nq; q++) {
        status[q] = oracle_graph2d(algo, occ, W, H, heuristic, starts[2 * q], starts[2 * q + 1], goals[2 * q],
                                   goals[2 * q + 1], &cost[q], path + (int64_t)q * path_cap, path_cap,
                                   &path_len[q], NULL, 0, &n_expanded[q], counters ? counters + 4 * (int64_t)q : NULL);
        found += status[q] == 0;
    }
    return found;
}

int oracle_astar2d_batch(const uint8_t* occ, int W, int H, int heuristic, const int32_t* starts,
                         const int32_t* goals, int nq, double* cost, int32_t* path, int path_cap,
                         int32_t* path_len, int32_t* n_expanded, int64_t* counters, int32_t* status,
                         int nthreads)
{
    return oracle_graph2d_batch(0, occ, W, H, heuristic, starts, goals, nq, cost, path, path_cap, path_len, n_expanded,
                                counters, status, nthreads);
}

/* ==================================================================================== */
/* Local planners (local_planner/ of the reference)                                      */
/* ==================================================================================== */

/* LocalPlanner.params (local_planner/local_planner.py:39-55), in this order */
typedef struct {
    double dt, lookahead_time, max_lookahead, min_lookahead, max_v_inc, min_v_inc, max_v, min_v,
        max_w_inc, min_w_inc, max_w, min_w, goal_dist_tol, rotate_tol;
} lp_params_t;

static const double PI_ = 3.141592653589793;

/* numpy pairwise summation (numpy/_core/src/umath/loops_utils.h pairwise_sum) over one buffer */
static double np_pairwise(const double* a, int64_t n, int64_t stride)
{
    if (n < 8) {
        double res = 0.0;
        for (int64_t i = 0; i < n; i++) res += a[i * stride];
        return res;
    } else if (n <= 128) {
        double r[8];
        int64_t i;
        for (int j = 0; j < 8; j++) r[j] = a[j * stride];
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += a[(i + j) * stride];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i * stride];
        return res;
    } else {
        int64_t n2 = n / 2;
        n2 -= n2 % 8;
        return np_pairwise(a, n2, stride) + np_pairwise(a + n2 * stride, n - n2, stride);
    }
}

/* np.sum of a strided 1-D view: pairwise per 8192-element buffer, buffers added in order */
double oracle_np_sum(const double* a, int64_t n, int64_t stride)
{
    double res = 0.0;
    for (int64_t i = 0; i < n; i += 8192) {
        int64_t m = n - i < 8192 ? n - i : 8192;
        res += np_pairwise(a + i * stride, m, stride);
    }
    return res;
}

/* np.linspace(a, b, num) (numpy/_core/function_base.py): i*step + a, last element = b */
static void np_linspace(double a, double b, int64_t num, double* out)
{
    if (num <= 0) return;
    if (num == 1) { out[0] = a; return; }
    const double div = (double)(num - 1), delta = b - a, step = delta / div;
    for (int64_t i = 0; i < num; i++) out[i] = (step == 0.0) ? ((double)i / div) * delta + a : (double)i * step + a;
    out[num - 1] = b;
}

static double regularize_angle(double a) { return a - 2.0 * PI_ * floor((a + PI_) / (2.0 * PI_)); }

static double clampd(double v, double lo, double hi)
{
    if (v < lo) v = lo;
    if (v > hi) v = hi;
    return v;
}

/* LocalPlanner.reachGoal (local_planner.py:233-246) */
int oracle_reach_goal(const double cur[3], const double goal[3], const lp_params_t* P)
{
    double e_theta = regularize_angle(cur[2] - goal[2]);
    int move = vnorm2(goal[0] - cur[0], goal[1] - cur[1]) > P->goal_dist_tol;
    int rot = fabs(e_theta) > P->rotate_tol;
    return !(move || rot);
}

/* LocalPlanner.getLookaheadPoint (local_planner.py:103-170) with MathHelper
 * (utils/helper/math_helper.py:11-65).  path: [P][2] start->goal.  robot: px, py, v.
 * Returns 0, or 4 where the reference raises (math domain error / index error). */
int oracle_lookahead(const double* path, int P, const double robot[3], const lp_params_t* Pr, double pt[2],
                     double* theta, double* kappa)
{
    const double rx = robot[0], ry = robot[1];
    const double L = clampd(fabs(robot[2]) * Pr->lookahead_time, Pr->min_lookahead, Pr->max_lookahead);
    if (P < 1) return 4;
    int idx_closest = 0;
    double best = vnorm2(rx - path[0], ry - path[1]);
    for (int i = 1; i < P; i++) {
        double d = vnorm2(rx - path[2 * i], ry - path[2 * i + 1]);
        if (d < best) { best = d; idx_closest = i; }
    }
    int idx_goal = P - 1, idx_prev = idx_goal - 1;
    for (int i = idx_closest; i < P; i++) {
        if (vnorm2(rx - path[2 * i], ry - path[2 * i + 1]) >= L) { idx_goal = i; break; }
    }
#define PX(i) path[2 * (((i) % P + P) % P)]
#define PY(i) path[2 * (((i) % P + P) % P) + 1]
    if (idx_goal == P - 1) {
        pt[0] = PX(idx_goal);
        pt[1] = PY(idx_goal);
    } else {
        if (idx_goal == 0) idx_goal = idx_goal + 1;
        idx_prev = idx_goal - 1;
        const double x1 = PX(idx_prev) - rx, y1 = PY(idx_prev) - ry;
        const double x2 = PX(idx_goal) - rx, y2 = PY(idx_goal) - ry;
        /* circleSegmentIntersection(prev_p, goal_p, L) */
        const double dx = x2 - x1, dy = y2 - y1;
        const double dr2 = dx * dx + dy * dy;
        const double D = x1 * y2 - x2 * y1;
        const double d1 = x1 * x1 + y1 * y1, d2 = x2 * x2 + y2 * y2, dd = d2 - d1;
        const double delta_2 = L * L * dr2 - D * D;
        double ix, iy;
        if (delta_2 < 0) {
            /* closestPointOnLine(prev_p, goal_p) */
            const double apx = 0.0 - x1, apy = 0.0 - y1, abx = x2 - x1, aby = y2 - y1;
            const double af = (apx * abx + apy * aby) / (abx * abx + aby * aby);
            ix = x1 + af * abx;
            iy = y1 + af * aby;
        } else {
            const double delta = sqrt(delta_2);
            if (delta == 0) {
                ix = D * dy / dr2;
                iy = -D * dx / dr2;
            } else {
                const double s = copysign(1.0, dd);
                ix = (D * dy + s * dx * delta) / dr2;
                iy = (-D * dx + s * dy * delta) / dr2;
            }
        }
        pt[0] = ix + rx;
        pt[1] = iy + ry;
    }
    if (idx_prev < -P || idx_goal >= P) return 4;
    *theta = atan2(PY(idx_goal) - PY(idx_prev), PX(idx_goal) - PX(idx_prev));
    if (idx_goal == 1) idx_goal = idx_goal + 1;
    if (idx_goal >= P) return 4; /* IndexError */
    idx_prev = idx_goal - 1;
    int idx_pprev = idx_prev - 1;
    const double a = vnorm2(PX(idx_goal) - PX(idx_prev), PY(idx_goal) - PY(idx_prev));
    const double b = vnorm2(PX(idx_goal) - PX(idx_pprev), PY(idx_goal) - PY(idx_pprev));
    const double c = vnorm2(PX(idx_prev) - PX(idx_pprev), PY(idx_prev) - PY(idx_pprev));
    if (a == 0.0 || c == 0.0 || b == 0.0) return 4; /* ZeroDivisionError */
    const double cosB = (a * a + c * c - b * b) / (2 * a * c);
    if (cosB > 1.0 || cosB < -1.0) return 4; /* math domain error */
    const double sinB = sin(acos(cosB));
    const double cross = (PX(idx_prev) - PX(idx_pprev)) * (PY(idx_goal) - PY(idx_pprev)) -
                         (PY(idx_prev) - PY(idx_pprev)) * (PX(idx_goal) - PX(idx_pprev));
    *kappa = copysign(2 * sinB / b, cross);
#undef PX
#undef PY
    return 0;
}

/* DWA.calDynamicWin (dwa.py:111-135) */
void oracle_dwa_window(double v, double w, const lp_params_t* P, double vr[4])
{
    const double vd0 = v + P->min_v_inc * P->dt, vd1 = v + P->max_v_inc * P->dt;
    const double vd2 = w + P->min_w_inc * P->dt, vd3 = w + P->max_w_inc * P->dt;
    vr[0] = fmax(P->min_v, vd0);
    vr[1] = fmin(P->max_v, vd1);
    vr[2] = fmax(P->min_w, vd2);
    vr[3] = fmin(P->max_w, vd3);
}

/* DWA.evaluation (dwa.py:137-190) + generateTraj (:192-212) + Robot.lookforward (agent.py:91-116).
 * obs: [nobs][2] (integer obstacle cells as doubles).  nv/nw > 0 override int((v1-v0)/v_res).
 * out: eval3 [N][3] = eval_win @ factor (v, w, score); best = argmax; best_traj [H][5].
 * Returns N (0 = the reference would raise on the empty window). */
/* Optional stencil form of the obstacle term (CPU-baseline variant, not the reference's loop): with a
 * grid set, min(min cdist(obstacles, traj), R) is taken over the occupied cells within R of each
 * trajectory point instead of over every obstacle.  Only cells with |dx|, |dy| <= R can be closer
 * than R, and min(sqrt(d2)) == sqrt(min(d2)), so the result is identical.  Set before a batch,
 * read-only during it; oracle_dwa_set_grid(NULL, ...) restores the brute-force loop. */
static const uint8_t* g_dwa_grid = NULL;
static int g_dwa_W = 0, g_dwa_H = 0;
void oracle_dwa_set_grid(const uint8_t* occ, int W, int H)
{
    g_dwa_grid = occ;
    g_dwa_W = W;
    g_dwa_H = H;
}

static double dwa_stencil_d2(double x, double y, double R, double mind2)
{
    const int x0 = (int)ceil(x - R), x1 = (int)floor(x + R), y0 = (int)ceil(y - R), y1 = (int)floor(y + R);
    for (int cx = x0 < 0 ? 0 : x0; cx <= x1 && cx < g_dwa_W; cx++)
        for (int cy = y0 < 0 ? 0 : y0; cy <= y1 && cy < g_dwa_H; cy++)
            if (g_dwa_grid[(size_t)cx * g_dwa_H + cy]) {
                const double dx = (double)cx - x, dy = (double)cy - y;
                const double d2 = dx * dx + dy * dy;
                if (d2 < mind2) mind2 = d2;
            }
    return mind2;
}

int oracle_dwa_eval(const double* obs, int nobs, const double st[5], const double goal[2], const double vr[4],
                    double v_res, double w_res, int nv, int nw, double predict_time, double dt, double hw,
                    double ow, double vw, double R, double* eval3, int* best, double* best_traj)
{
    if (nv <= 0) nv = (int)((vr[1] - vr[0]) / v_res);
    if (nw <= 0) nw = (int)((vr[3] - vr[2]) / w_res);
    const int N = nv * nw, H = (int)(predict_time / dt);
    if (N <= 0 || nv < 0 || nw < 0) return 0;
    double* vs = (double*)malloc(sizeof(double) * (size_t)nv);
    double* ws = (double*)malloc(sizeof(double) * (size_t)nw);
    double* ew = (double*)malloc(sizeof(double) * (size_t)N * 5);
    np_linspace(vr[0], vr[1], nv, vs);
    np_linspace(vr[2], vr[3], nw, ws);
    for (int c = 0; c < N; c++) {
        const double v = vs[c / nw], w = ws[c % nw];
        double x = st[0], y = st[1], th = st[2];
        double mind = INFINITY, mind2 = INFINITY;
        for (int k = 0; k < H; k++) {
            const double nx = x + (dt * cos(th)) * v, ny = y + (dt * sin(th)) * v, nth = th + dt * w;
            x = nx; y = ny; th = nth;
            if (g_dwa_grid) {
                mind2 = dwa_stencil_d2(x, y, R, mind2);
                continue;
            }
            for (int o = 0; o < nobs; o++) {
                const double dx = obs[2 * o] - x, dy = obs[2 * o + 1] - y;
                const double d = sqrt(dx * dx + dy * dy);
                if (d < mind) mind = d;
            }
        }
        if (g_dwa_grid) mind = sqrt(mind2);
        const double theta = atan2(goal[1] - y, goal[0] - x);
        ew[5 * c + 0] = v;
        ew[5 * c + 1] = w;
        ew[5 * c + 2] = PI_ - fabs(theta - th);
        ew[5 * c + 3] = mind < R ? mind : R; /* min(min_D, R): min_D kept on ties, same value */
        ew[5 * c + 4] = fabs(v);
    }
    for (int col = 2; col < 5; col++) {
        const double s = oracle_np_sum(ew + col, N, 5);
        if (s != 0)
            for (int c = 0; c < N; c++) ew[5 * c + col] = ew[5 * c + col] / s;
    }
    int bi = 0;
    double bs = -INFINITY;
    for (int c = 0; c < N; c++) {
        const double* e = ew + 5 * c;
        /* (eval_win @ factor) on OpenBLAS: a k-ordered fma chain per output element */
        const double c0 = fma(e[4], 0.0, fma(e[3], 0.0, fma(e[2], 0.0, fma(e[1], 0.0, e[0] * 1.0))));
        const double c1 = fma(e[4], 0.0, fma(e[3], 0.0, fma(e[2], 0.0, fma(e[1], 1.0, e[0] * 0.0))));
        const double c2 = fma(e[4], vw, fma(e[3], ow, fma(e[2], hw, fma(e[1], 0.0, e[0] * 0.0))));
        if (eval3) { eval3[3 * c] = c0; eval3[3 * c + 1] = c1; eval3[3 * c + 2] = c2; }
        if (c2 > bs || c == 0) { bs = c2; bi = c; }
    }
    *best = bi;
    if (best_traj) {
        const double v = vs[bi / nw], w = ws[bi % nw];
        double x = st[0], y = st[1], th = st[2];
        for (int k = 0; k < H; k++) {
            const double nx = x + (dt * cos(th)) * v, ny = y + (dt * sin(th)) * v, nth = th + dt * w;
            x = nx; y = ny; th = nth;
            best_traj[5 * k] = x; best_traj[5 * k + 1] = y; best_traj[5 * k + 2] = th;
            best_traj[5 * k + 3] = v; best_traj[5 * k + 4] = w;
        }
    }
    free(vs); free(ws); free(ew);
    return N;
}

/* one DWA.plan iteration (dwa.py:72-93).  st[5] updated in place.  Returns 0 stepped, 1 goal
 * reached (no step), 4 the reference raises (empty window / lookahead error). */
int oracle_dwa_step(const double* obs, int nobs, const double* path, int P, const double goal[3], double st[5],
                    const lp_params_t* Pr, double v_res, double w_res, int nv, int nw, double predict_time,
                    double hw, double ow, double vw, double R, double u[2])
{
    const double cur[3] = {st[0], st[1], st[2]};
    if (oracle_reach_goal(cur, goal, Pr)) return 1;
    double pt[2], theta, kappa;
    const double rob[3] = {st[0], st[1], st[3]};
    if (oracle_lookahead(path, P, rob, Pr, pt, &theta, &kappa)) return 4;
    double vr[4];
    oracle_dwa_window(st[3], st[4], Pr, vr);
    int best;
    double* e3 = NULL;
    int n = oracle_dwa_eval(obs, nobs, st, pt, vr, v_res, w_res, nv, nw, predict_time, Pr->dt, hw, ow, vw, R, e3, &best, NULL);
    if (n <= 0) return 4;
    /* recompute the chosen (v, w) exactly as evaluation's linspace produced them */
    if (nv <= 0) nv = (int)((vr[1] - vr[0]) / v_res);
    if (nw <= 0) nw = (int)((vr[3] - vr[2]) / w_res);
    double* vs = (double*)malloc(sizeof(double) * (size_t)nv);
    double* ws = (double*)malloc(sizeof(double) * (size_t)nw);
    np_linspace(vr[0], vr[1], nv, vs);
    np_linspace(vr[2], vr[3], nw, ws);
    u[0] = vs[best / nw];
    u[1] = ws[best % nw];
    free(vs); free(ws);
    /* Robot.kinematic -> lookforward(state, u, dt) */
    const double dt = Pr->dt;
    const double nx = st[0] + (dt * cos(st[2])) * u[0], ny = st[1] + (dt * sin(st[2])) * u[0];
    const double nth = st[2] + dt * u[1];
    st[0] = nx; st[1] = ny; st[2] = nth; st[3] = u[0]; st[4] = u[1];
    return 0;
}

/* LQR parameters (lqr.py:35-38): diag Q, diag R, Riccati iteration cap, signed exit threshold.
 * Layout mirrors pmp_lqr_params in include/pmp.h. */
typedef struct {
    double q[3], r[2];
    int32_t iters;
    double eps;
} lqr_params_t;

/* LQR.lqrControl (local_planner/lqr.py:103-145): discrete Riccati iteration with the signed
 * `max(P - P_) < eps` exit (:132-136), K = -(R + B'P_B)^-1 B'P_A (:139), u = u_r + K e (:140-141),
 * then linear/angular regularisation (local_planner.py:172-206) against the robot's current (v, w). */
void oracle_lqr_control(const double s[3], const double sd[3], const double ur[2], double rv, double rw,
                        const lp_params_t* Pr, const lqr_params_t* L, double u[2])
{
    const double dt = Pr->dt;
    double A[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}}, B[3][2] = {{0, 0}, {0, 0}, {0, 0}};
    A[0][2] = -ur[0] * sin(sd[2]) * dt;
    A[1][2] = ur[0] * cos(sd[2]) * dt;
    B[0][0] = cos(sd[2]) * dt;
    B[1][0] = sin(sd[2]) * dt;
    B[2][1] = dt;
    double Pm[3][3] = {{L->q[0], 0, 0}, {0, L->q[1], 0}, {0, 0, L->q[2]}}, Pn[3][3];
    memset(Pn, 0, sizeof(Pn));  /* P_ = zeros when the loop body never runs (lqr.py:128) */
    for (int it = 0; it < L->iters; it++) {
        double PA[3][3], PB[3][2], APA[3][3], APB[3][2], BPB[2][2], BPA[2][3], S[2][2], Si[2][2];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) { PA[i][j] = 0; for (int k = 0; k < 3; k++) PA[i][j] += Pm[i][k] * A[k][j]; }
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 2; j++) { PB[i][j] = 0; for (int k = 0; k < 3; k++) PB[i][j] += Pm[i][k] * B[k][j]; }
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) { APA[i][j] = 0; for (int k = 0; k < 3; k++) APA[i][j] += A[k][i] * PA[k][j]; }
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 2; j++) { APB[i][j] = 0; for (int k = 0; k < 3; k++) APB[i][j] += A[k][i] * PB[k][j]; }
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 2; j++) { BPB[i][j] = 0; for (int k = 0; k < 3; k++) BPB[i][j] += B[k][i] * PB[k][j]; }
        for (int i = 0; i < 2; i++)
            for (int j = 0; j < 3; j++) { BPA[i][j] = 0; for (int k = 0; k < 3; k++) BPA[i][j] += B[k][i] * PA[k][j]; }
        for (int i = 0; i < 2; i++) for (int j = 0; j < 2; j++) S[i][j] = (i == j ? L->r[i] : 0.0) + BPB[i][j];
        const double det = S[0][0] * S[1][1] - S[0][1] * S[1][0];
        Si[0][0] = S[1][1] / det; Si[0][1] = -S[0][1] / det; Si[1][0] = -S[1][0] / det; Si[1][1] = S[0][0] / det;
        double mx = -INFINITY;
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                double corr = 0;
                for (int a = 0; a < 2; a++)
                    for (int b = 0; b < 2; b++) corr += APB[i][a] * Si[a][b] * BPA[b][j];
                Pn[i][j] = (i == j ? L->q[i] : 0.0) + APA[i][j] - corr;
                if (Pm[i][j] - Pn[i][j] > mx) mx = Pm[i][j] - Pn[i][j];
            }
        if (mx < L->eps) break;
        memcpy(Pm, Pn, sizeof(Pm));
    }
    /* K = -(R + B'P_B)^-1 B'P_A with P_ the last update */
    double PB[3][2], PA[3][3], BPB[2][2], BPA[2][3], Si[2][2];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 2; j++) { PB[i][j] = 0; for (int k = 0; k < 3; k++) PB[i][j] += Pn[i][k] * B[k][j]; }
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) { PA[i][j] = 0; for (int k = 0; k < 3; k++) PA[i][j] += Pn[i][k] * A[k][j]; }
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 2; j++) { BPB[i][j] = (i == j ? L->r[i] : 0.0); for (int k = 0; k < 3; k++) BPB[i][j] += B[k][i] * PB[k][j]; }
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 3; j++) { BPA[i][j] = 0; for (int k = 0; k < 3; k++) BPA[i][j] += B[k][i] * PA[k][j]; }
    const double det = BPB[0][0] * BPB[1][1] - BPB[0][1] * BPB[1][0];
    Si[0][0] = BPB[1][1] / det; Si[0][1] = -BPB[0][1] / det; Si[1][0] = -BPB[1][0] / det; Si[1][1] = BPB[0][0] / det;
    double K[2][3];
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 3; j++) { K[i][j] = 0; for (int a = 0; a < 2; a++) K[i][j] -= Si[i][a] * BPA[a][j]; }
    const double e[3] = {s[0] - sd[0], s[1] - sd[1], regularize_angle(s[2] - sd[2])};
    double uu[2];
    for (int i = 0; i < 2; i++) { uu[i] = ur[i]; for (int j = 0; j < 3; j++) uu[i] += K[i][j] * e[j]; }
    /* linearRegularization / angularRegularization */
    double vi = clampd(uu[0] - rv, Pr->min_v_inc, Pr->max_v_inc);
    u[0] = clampd(rv + vi, Pr->min_v, Pr->max_v);
    double wi = clampd(uu[1] - rw, Pr->min_w_inc, Pr->max_w_inc);
    u[1] = clampd(rw + wi, Pr->min_w, Pr->max_w);
}

/* MPC parameters: horizons and weights of mpc.py:37-40, then the ADMM settings of the QP solve
 * (OSQP's defaults: rho 0.1, sigma 1e-6, alpha 1.6, eps 1e-3/1e-3, 4000 iterations, termination
 * checked every 25, rho adapted every 25 with tolerance 5).  Mirrors pmp_mpc_params. */
typedef struct {
    int32_t p, m;
    double q[3], r[2];
    double rho, sigma, alpha, eps_abs, eps_rel, adaptive_tol;
    int32_t max_iter, check_every, adaptive_every, reserved;
} mpc_params_t;

/* MPC.mpcControl QP assembly (mpc.py:124-200), written literally: A5/B5/C, S_x and S_u from
 * repeated products of A5 (np.linalg.matrix_power), H = S_u'QS_u + R, g = S_u'Q(S_x x - 0),
 * l/u of [kron(tril(1_m), I2); I_2m].  H [2m][2m], g [2m], l/u [4m]. */
void oracle_mpc_assemble(const double s[3], const double sd[3], const double ur[2], const double up[2],
                         const lp_params_t* Pr, const mpc_params_t* M, double* H, double* g, double* lo, double* hi)
{
    const int p = M->p, m = M->m, n = 2 * m;
    const double dt = Pr->dt;
    double A[5][5], B[5][2];
    memset(A, 0, sizeof(A));
    memset(B, 0, sizeof(B));
    for (int i = 0; i < 5; i++) A[i][i] = 1.0;
    A[0][2] = -ur[0] * sin(sd[2]) * dt;
    A[1][2] = ur[0] * cos(sd[2]) * dt;
    B[0][0] = cos(sd[2]) * dt;
    B[1][0] = sin(sd[2]) * dt;
    B[2][1] = dt;
    A[0][3] = B[0][0]; A[1][3] = B[1][0]; A[2][4] = B[2][1];  /* [[A, B], [0, I]] */
    B[3][0] = 1.0; B[4][1] = 1.0;                            /* [B; I] */
    const double x[5] = {s[0] - sd[0], s[1] - sd[1], s[2] - sd[2], up[0], up[1]};
    /* powers A^0 .. A^p (first three rows are all C A^k needs) */
    double (*Ap)[5][5] = (double (*)[5][5])malloc(sizeof(double) * 25 * (size_t)(p + 1));
    memset(Ap[0], 0, sizeof(Ap[0]));
    for (int i = 0; i < 5; i++) Ap[0][i][i] = 1.0;
    for (int k = 1; k <= p; k++)
        for (int i = 0; i < 5; i++)
            for (int j = 0; j < 5; j++) {
                double acc = 0;
                for (int t = 0; t < 5; t++) acc += Ap[k - 1][i][t] * A[t][j];
                Ap[k][i][j] = acc;
            }
    const int R3 = 3 * p;
    double* Su = (double*)calloc((size_t)R3 * n, sizeof(double));
    double* y = (double*)calloc((size_t)R3, sizeof(double));
    for (int i = 0; i < p; i++) {
        for (int d = 0; d < 3; d++) {
            double acc = 0;
            for (int t = 0; t < 5; t++) acc += Ap[i + 1][d][t] * x[t];
            y[3 * i + d] = acc;  /* (S_x x)_r ; Yr = 0 */
        }
        for (int j = 0; j < m && j <= i; j++)
            for (int d = 0; d < 3; d++)
                for (int c = 0; c < 2; c++) {
                    double acc = 0;
                    for (int t = 0; t < 5; t++) acc += Ap[i - j][d][t] * B[t][c];
                    Su[(size_t)(3 * i + d) * n + 2 * j + c] = acc;
                }
    }
    for (int a = 0; a < n; a++) {
        for (int b = 0; b < n; b++) {
            double acc = 0;
            for (int r = 0; r < R3; r++) acc += Su[(size_t)r * n + a] * M->q[r % 3] * Su[(size_t)r * n + b];
            H[a * n + b] = acc + (a == b ? M->r[a % 2] : 0.0);
        }
        double acc = 0;
        for (int r = 0; r < R3; r++) acc += Su[(size_t)r * n + a] * M->q[r % 3] * y[r];
        g[a] = acc;
    }
    for (int k = 0; k < m; k++) {
        lo[2 * k] = Pr->min_v - up[0];        hi[2 * k] = Pr->max_v - up[0];
        lo[2 * k + 1] = Pr->min_w - up[1];    hi[2 * k + 1] = Pr->max_w - up[1];
        lo[n + 2 * k] = Pr->min_v_inc;        hi[n + 2 * k] = Pr->max_v_inc;
        lo[n + 2 * k + 1] = Pr->min_w_inc;    hi[n + 2 * k + 1] = Pr->max_w_inc;
    }
    free(Ap); free(Su); free(y);
}

/* y = A x and x = A' y for A = [kron(tril(1_m), I2); I_2m] (mpc.py:185,197) */
static void mpc_Ax(int m, const double* x, double* Ax)
{
    const int n = 2 * m;
    double c0 = 0, c1 = 0;
    for (int k = 0; k < m; k++) {
        c0 += x[2 * k]; c1 += x[2 * k + 1];
        Ax[2 * k] = c0; Ax[2 * k + 1] = c1;
        Ax[n + 2 * k] = x[2 * k]; Ax[n + 2 * k + 1] = x[2 * k + 1];
    }
}

static void mpc_ATy(int m, const double* y, double* ATy)
{
    const int n = 2 * m;
    double c0 = 0, c1 = 0;
    for (int k = m - 1; k >= 0; k--) {
        c0 += y[2 * k]; c1 += y[2 * k + 1];
        ATy[2 * k] = c0 + y[n + 2 * k];
        ATy[2 * k + 1] = c1 + y[n + 2 * k + 1];
    }
}

/* Cholesky of K = H + sigma I + rho A'A (A'A[2k+c][2k'+c] = m - max(k, k'), plus I) */
static void mpc_factor(int m, const double* H, double sigma, double rho, double* Lc)
{
    const int n = 2 * m;
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
            const int ki = i / 2, kj = j / 2;
            double t = (i % 2 == j % 2) ? (double)(m - (ki > kj ? ki : kj)) : 0.0;
            Lc[i * n + j] = H[i * n + j] + rho * (t + (i == j ? 1.0 : 0.0)) + (i == j ? sigma : 0.0);
        }
    for (int j = 0; j < n; j++) {
        double d = Lc[j * n + j];
        for (int k = 0; k < j; k++) d -= Lc[j * n + k] * Lc[j * n + k];
        d = sqrt(d);
        Lc[j * n + j] = d;
        for (int i = j + 1; i < n; i++) {
            double v = Lc[i * n + j];
            for (int k = 0; k < j; k++) v -= Lc[i * n + k] * Lc[j * n + k];
            Lc[i * n + j] = v / d;
        }
    }
}

static void mpc_solve(int n, const double* Lc, double* b)
{
    for (int i = 0; i < n; i++) {
        double v = b[i];
        for (int k = 0; k < i; k++) v -= Lc[i * n + k] * b[k];
        b[i] = v / Lc[i * n + i];
    }
    for (int i = n - 1; i >= 0; i--) {
        double v = b[i];
        for (int k = i + 1; k < n; k++) v -= Lc[k * n + i] * b[k];
        b[i] = v / Lc[i * n + i];
    }
}

static double inf_norm(const double* v, int n)
{
    double r = 0;
    for (int i = 0; i < n; i++) r = fabs(v[i]) > r ? fabs(v[i]) : r;
    return r;
}

/* The QP solve of mpc.py:196-203: min 1/2 x'Hx + g'x s.t. lo <= A x <= hi, by OSQP's ADMM
 * (x~ from the reduced KKT system, relaxation alpha, projection onto [lo, hi], dual update,
 * termination on the unscaled inf-norm residuals, rho adaptation by the residual ratio).  OSQP
 * itself is not installed here: this restates its published algorithm without Ruiz scaling or
 * polishing (parity with OSQP's bits is unpinned; the optimum is pinned by KKT checks).
 * Returns 0 converged, 1 iteration limit.  *iters = iterations run, *rho_out = final rho. */
int oracle_qp_admm(int m, const double* H, const double* g, const double* lo, const double* hi,
                   const mpc_params_t* M, double* x, int* iters, double* rho_out)
{
    const int n = 2 * m, nc = 4 * m;
    double Lc[256], z[32], y[32], rhs[16], w[32], xt[16], zt[32], Ax[32], ATy[16], Hx[16], r[32];
    double rho = M->rho;
    const double sigma = M->sigma, alpha = M->alpha;
    for (int i = 0; i < n; i++) x[i] = 0;
    for (int i = 0; i < nc; i++) z[i] = y[i] = 0;
    mpc_factor(m, H, sigma, rho, Lc);
    int status = 1, it;
    for (it = 1; it <= M->max_iter; it++) {
        const double rinv = 1.0 / rho;
        for (int i = 0; i < nc; i++) w[i] = rho * z[i] - y[i];
        mpc_ATy(m, w, rhs);
        for (int i = 0; i < n; i++) rhs[i] = sigma * x[i] - g[i] + rhs[i];
        mpc_solve(n, Lc, rhs);
        for (int i = 0; i < n; i++) xt[i] = rhs[i];
        mpc_Ax(m, xt, zt);
        for (int i = 0; i < n; i++) x[i] = alpha * xt[i] + (1.0 - alpha) * x[i];
        for (int i = 0; i < nc; i++) {
            const double zr = alpha * zt[i] + (1.0 - alpha) * z[i];
            const double zn = clampd(zr + rinv * y[i], lo[i], hi[i]);
            y[i] = y[i] + rho * (zr - zn);
            z[i] = zn;
        }
        const int check = (M->check_every > 0 && it % M->check_every == 0) || it == M->max_iter;
        const int adapt = M->adaptive_every > 0 && it % M->adaptive_every == 0;
        if (!check && !adapt) continue;
        mpc_Ax(m, x, Ax);
        mpc_ATy(m, y, ATy);
        for (int i = 0; i < n; i++) {
            double acc = 0;
            for (int j = 0; j < n; j++) acc += H[i * n + j] * x[j];
            Hx[i] = acc;
        }
        for (int i = 0; i < nc; i++) r[i] = Ax[i] - z[i];
        const double prim = inf_norm(r, nc);
        for (int i = 0; i < n; i++) rhs[i] = Hx[i] + g[i] + ATy[i];
        const double dual = inf_norm(rhs, n);
        const double nAx = inf_norm(Ax, nc), nz = inf_norm(z, nc);
        const double nHx = inf_norm(Hx, n), nATy = inf_norm(ATy, n), ng = inf_norm(g, n);
        const double pscale = nAx > nz ? nAx : nz;
        double dscale = nHx > nATy ? nHx : nATy;
        dscale = dscale > ng ? dscale : ng;
        if (check && prim <= M->eps_abs + M->eps_rel * pscale && dual <= M->eps_abs + M->eps_rel * dscale) {
            status = 0;
            break;
        }
        if (adapt) {
            const double pn = prim / (pscale + 1e-30), dn = dual / (dscale + 1e-30);
            double rn = rho * sqrt(pn / (dn + 1e-30));
            rn = clampd(rn, 1e-6, 1e6);
            if (rn > rho * M->adaptive_tol || rn < rho / M->adaptive_tol) {
                rho = rn;
                mpc_factor(m, H, sigma, rho, Lc);
            }
        }
    }
    if (iters) *iters = it > M->max_iter ? M->max_iter : it;
    if (rho_out) *rho_out = rho;
    return status;
}

/* MPC.mpcControl (mpc.py:111-214): assemble, solve, u = du0 + u_p + u_r, regularise; returns the
 * new u_p = u - u_r (before regularisation).  Returns the ADMM status; *iters as above. */
int oracle_mpc_control(const double s[3], const double sd[3], const double ur[2], double up[2], double rv, double rw,
                       const lp_params_t* Pr, const mpc_params_t* M, double u[2], int* iters)
{
    double H[256], g[16], lo[32], hi[32], x[16];
    oracle_mpc_assemble(s, sd, ur, up, Pr, M, H, g, lo, hi);
    const int st = oracle_qp_admm(M->m, H, g, lo, hi, M, x, iters, NULL);
    const double uu0 = (x[0] + up[0]) + ur[0], uu1 = (x[1] + up[1]) + ur[1];
    up[0] = uu0 - ur[0];
    up[1] = uu1 - ur[1];
    const double vi = clampd(uu0 - rv, Pr->min_v_inc, Pr->max_v_inc);
    u[0] = clampd(rv + vi, Pr->min_v, Pr->max_v);
    const double wi = clampd(uu1 - rw, Pr->min_w_inc, Pr->max_w_inc);
    u[1] = clampd(rw + wi, Pr->min_w, Pr->max_w);
    return st;
}

/* One LQR.plan (lqr.py:58-86) or MPC.plan (mpc.py:66-94) iteration: kind 0 = LQR, 1 = MPC.
 * st[5] = (x, y, theta, v, w) updated in place; up[2] is MPC's carried u_p.  Returns 0 stepped,
 * 1 goal reached (no step), 4 the reference raises (getLookaheadPoint). */
int oracle_track_step(int kind, const double* path, int P, const double goal[3], double st[5], double up[2],
                      const lp_params_t* Pr, const lqr_params_t* L, const mpc_params_t* M, double u[2], int* admm_iters)
{
    const double cur[3] = {st[0], st[1], st[2]};
    if (admm_iters) *admm_iters = 0;
    if (oracle_reach_goal(cur, goal, Pr)) return 1;
    double pt[2], theta, kappa;
    const double rob[3] = {st[0], st[1], st[3]};
    if (oracle_lookahead(path, P, rob, Pr, pt, &theta, &kappa)) return 4;
    const double dt = Pr->dt;
    double e_theta = regularize_angle(st[2] - goal[2]);
    /* angularRegularization(w_d) against the current w */
#define ANGREG(wd) clampd(st[4] + clampd((wd) - st[4], Pr->min_w_inc, Pr->max_w_inc), Pr->min_w, Pr->max_w)
    if (!(vnorm2(goal[0] - st[0], goal[1] - st[1]) > Pr->goal_dist_tol)) {
        u[0] = 0.0;
        u[1] = (fabs(e_theta) > Pr->rotate_tol) ? ANGREG(e_theta / dt) : 0.0;
    } else {
        e_theta = regularize_angle(atan2(pt[1] - st[1], pt[0] - st[0]) - st[2]);
        if (fabs(e_theta) > Pr->rotate_tol) {
            u[0] = 0.0;
            u[1] = ANGREG(e_theta / dt);
        } else {
            const double s[3] = {st[0], st[1], st[2]}, sd[3] = {pt[0], pt[1], theta};
            const double ur[2] = {st[3], st[3] * kappa};
            if (kind == 0)
                oracle_lqr_control(s, sd, ur, st[3], st[4], Pr, L, u);
            else
                oracle_mpc_control(s, sd, ur, up, st[3], st[4], Pr, M, u, admm_iters);
        }
    }
#undef ANGREG
    /* Robot.kinematic -> lookforward (agent.py:68-116) */
    const double nx = st[0] + (dt * cos(st[2])) * u[0], ny = st[1] + (dt * sin(st[2])) * u[0];
    const double nth = st[2] + dt * u[1];
    st[0] = nx; st[1] = ny; st[2] = nth; st[3] = u[0]; st[4] = u[1];
    return 0;
}

/* OpenMP over agents: `iters` plan iterations each (stops at the first non-zero status).
 * Returns the number of agent-steps taken. */
int64_t oracle_track_batch(int kind, const double* path_xy, const int32_t* path_off, const double* goals, double* st,
                           double* up, int na, int iters, const lp_params_t* Pr, const lqr_params_t* L,
                           const mpc_params_t* M, double* u, int32_t* status, int32_t* n_steps, int nthreads)
{
    int64_t total = 0;
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) reduction(+ : total)
    for (int a = 0; a < na; a++) {
        int rc = 0, k;
        for (k = 0; k < iters; k++) {
            rc = oracle_track_step(kind, path_xy + 2 * (int64_t)path_off[a], path_off[a + 1] - path_off[a], goals + 3 * a,
                                   st + 5 * a, up + 2 * a, Pr, L, M, u + 2 * a, NULL);
            if (rc) break;
        }
        status[a] = rc;
        n_steps[a] = k;
        total += k;
    }
    return total;
}

/* OpenMP over agents: one DWA.plan iteration for each (CPU baseline of bench.py's control leg).
 * paths: path_xy [*][2] + path_off [na+1]; st [na][5] updated; u [na][2]; returns # stepped. */
int oracle_dwa_step_batch(const double* obs, int nobs, const double* path_xy, const int32_t* path_off,
                          const double* goals, double* st, int na, const lp_params_t* Pr, double v_res,
                          double w_res, int nv, int nw, double predict_time, double hw, double ow, double vw,
                          double R, double* u, int32_t* status, int nthreads)
{
    int stepped = 0;
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) reduction(+ : stepped)
    for (int a = 0; a < na; a++) {
        status[a] = oracle_dwa_step(obs, nobs, path_xy + 2 * (int64_t)path_off[a], path_off[a + 1] - path_off[a],
                                    goals + 3 * a, st + 5 * a, Pr, v_res, w_res, nv, nw, predict_time, hw, ow, vw,
                                    R, u + 2 * a);
        stepped += status[a] == 0;
    }
    return stepped;
}

/* ==================================================================================== */
/* Sample search: RRT / RRT* over a Map (global_planner/sample_search/)                  */
/* ==================================================================================== */

/* Map obstacles: rects [nr][4] (ox, oy, w, h), circles [nc][3] (ox, oy, r), boundary [nb][4]
 * (utils/environment/env.py:83-117), inflation delta (sample_search.py:22-25). */
typedef struct {
    const double *rect, *circ, *bnd;
    int nr, nc, nb;
    double delta;
} map_t;

/* SampleSearcher.isInsideObs (sample_search.py:51-77) */
static int map_inside(const map_t* M, double x, double y)
{
    const double d = M->delta;
    for (int i = 0; i < M->nc; i++) {
        const double* c = M->circ + 3 * i;
        if (vnorm2(x - c[0], y - c[1]) <= c[2] + d) return 1;
    }
    for (int i = 0; i < M->nr; i++) {
        const double* r = M->rect + 4 * i;
        const double px = x - (r[0] - d), py = y - (r[1] - d);
        if (0 <= px && px <= r[2] + 2 * d && 0 <= py && py <= r[3] + 2 * d) return 1;
    }
    for (int i = 0; i < M->nb; i++) {
        const double* r = M->bnd + 4 * i;
        const double px = x - (r[0] - d), py = y - (r[1] - d);
        if (0 <= px && px <= r[2] + 2 * d && 0 <= py && py <= r[3] + 2 * d) return 1;
    }
    return 0;
}

static double cross3(double p1x, double p1y, double p2x, double p2y, double p3x, double p3y)
{
    const double x1 = p2x - p1x, y1 = p2y - p1y, x2 = p3x - p1x, y2 = p3y - p1y;
    return x1 * y2 - x2 * y1;
}

/* SampleSearcher.isInterRect (sample_search.py:79-109): all 6 vertex pairs of the inflated rect
 * (itertools.combinations order), bbox "rapid repulsion" then the straddle test. */
static int map_inter_rect(const double* r, double d, double x1, double y1, double x2, double y2)
{
    const double vx[4] = {r[0] - d, r[0] + r[2] + d, r[0] + r[2] + d, r[0] - d};
    const double vy[4] = {r[1] - d, r[1] - d, r[1] + r[3] + d, r[1] + r[3] + d};
    for (int a = 0; a < 4; a++)
        for (int b = a + 1; b < 4; b++) {
            if (fmax(x1, x2) >= fmin(vx[a], vx[b]) && fmin(x1, x2) <= fmax(vx[a], vx[b]) &&
                fmax(y1, y2) >= fmin(vy[a], vy[b]) && fmin(y1, y2) <= fmax(vy[a], vy[b])) {
                if (cross3(vx[a], vy[a], vx[b], vy[b], x1, y1) * cross3(vx[a], vy[a], vx[b], vy[b], x2, y2) <= 0 &&
                    cross3(x1, y1, x2, y2, vx[a], vy[a]) * cross3(x1, y1, x2, y2, vx[b], vy[b]) <= 0)
                    return 1;
            }
        }
    return 0;
}

/* SampleSearcher.isInterCircle (sample_search.py:111-135).  np.dot of two 2-vectors is OpenBLAS
 * ddot, whose scalar tail accumulates with FMA: dot = fma(a1, b1, a0 * b0). */
static int map_inter_circle(const double* c, double d, double x, double y, double x2, double y2)
{
    const double dx = x2 - x, dy = y2 - y;
    const double d2 = fma(dy, dy, dx * dx);
    if (d2 == 0) return 0;
    const double t = fma(c[1] - y, dy, (c[0] - x) * dx) / d2;
    if (0 <= t && t <= 1) {
        const double sx = x + t * dx, sy = y + t * dy;
        if (vnorm2(c[0] - sx, c[1] - sy) <= c[2] + d) return 1;
    }
    return 0;
}

/* SampleSearcher.isCollision(node1, node2) (sample_search.py:27-49); argument order matters */
static int map_collision(const map_t* M, double x1, double y1, double x2, double y2)
{
    if (map_inside(M, x1, y1) || map_inside(M, x2, y2)) return 1;
    for (int i = 0; i < M->nr; i++)
        if (map_inter_rect(M->rect + 4 * i, M->delta, x1, y1, x2, y2)) return 1;
    for (int i = 0; i < M->nc; i++)
        if (map_inter_circle(M->circ + 3 * i, M->delta, x1, y1, x2, y2)) return 1;
    return 0;
}

int oracle_map_collision(const double* rect, int nr, const double* circ, int nc, const double* bnd, int nb,
                         double delta, double x1, double y1, double x2, double y2)
{
    const map_t M = {rect, circ, bnd, nr, nc, nb, delta};
    return map_collision(&M, x1, y1, x2, y2);
}

/* RRT.plan (rrt.py:49-83) with RRT.getNearest (rrt.py:105-130) or RRTStar.getNearest
 * (rrt_star.py:43-76).  rnd: the np.random double stream (RandomState.random_sample order) that
 * generateRandomNode (rrt.py:91-103) consumes: one draw, then two uniforms when it exceeds
 * goal_rate.  The sample_list dict is the tree array in insertion order; a node whose
 * coordinates already exist replaces that entry in place (dict semantics).
 * tree [cap][4] = x, y, g, parent index (the start is its own parent, node.py:33).  Returns 0 found, 1 not found,
 * 3 capacity / random-stream overflow.  *n_nodes includes the goal when found; *draws = doubles
 * consumed. */
int oracle_rrt(int star, const double* rect, int nr, const double* circ, int nc, const double* bnd, int nb,
               double delta, double X, double Y, double sx, double sy, double gx, double gy, int sample_num,
               double max_dist, double radius, double goal_rate, const double* rnd, int64_t nrnd, double* tree,
               int cap, int* n_nodes, int64_t* draws)
{
    const map_t M = {rect, circ, bnd, nr, nc, nb, delta};
    const double lox = delta, rgx = (X - delta) - delta, loy = delta, rgy = (Y - delta) - delta;
    int n = 1, status = 1;
    int64_t cur = 0;
    tree[0] = sx; tree[1] = sy; tree[2] = 0.0; tree[3] = 0;  /* start.parent = start.current */
    for (int it = 0; it < sample_num; it++) {
        if (cur + 3 > nrnd) { status = 3; break; }
        double rx = gx, ry = gy;
        if (rnd[cur++] > goal_rate) {
            rx = lox + rgx * rnd[cur++];
            ry = loy + rgy * rnd[cur++];
        }
        int dup = 0, bi = 0;
        double best = INFINITY;
        for (int j = 0; j < n; j++) {
            const double* t = tree + 4 * j;
            if (t[0] == rx && t[1] == ry) dup = 1;
            const double d = vnorm2(rx - t[0], ry - t[1]);
            if (d < best) { best = d; bi = j; }
        }
        if (dup) continue;
        const double* near = tree + 4 * bi;
        double dist = vnorm2(rx - near[0], ry - near[1]);
        const double theta = atan2(ry - near[1], rx - near[0]);
        if (max_dist < dist) dist = max_dist;  /* min(self.max_dist, dist) */
        const double nx = near[0] + dist * cos(theta), ny = near[1] + dist * sin(theta);
        double g = near[2] + dist;
        int parent = bi;
        if (map_collision(&M, nx, ny, near[0], near[1])) continue;
        /* where does node_new land in the dict? */
        int slot = n;
        if (star) {
            for (int j = 0; j < n; j++)
                if (tree[4 * j] == nx && tree[4 * j + 1] == ny) { slot = j; break; }
            for (int j = 0; j < n; j++) {
                double* t = tree + 4 * j;
                const double d = vnorm2(nx - t[0], ny - t[1]);
                if (!(d < radius)) continue;
                const double c = t[2] + d;
                if (g > c && !map_collision(&M, t[0], t[1], nx, ny)) {
                    parent = j;
                    g = c;
                } else {
                    const double c2 = g + d;
                    if (t[2] > c2 && !map_collision(&M, t[0], t[1], nx, ny)) {
                        t[3] = slot;
                        t[2] = c2;
                    }
                }
            }
        } else {
            for (int j = 0; j < n; j++)
                if (tree[4 * j] == nx && tree[4 * j + 1] == ny) { slot = j; break; }
        }
        if (slot == n) {
            if (n >= cap) { status = 3; break; }
            n++;
        }
        double* t = tree + 4 * slot;
        t[0] = nx; t[1] = ny; t[2] = g; t[3] = parent;
        const double dg = vnorm2(gx - nx, gy - ny);
        if (dg <= max_dist && !map_collision(&M, nx, ny, gx, gy)) {
            if (n >= cap) { status = 3; break; }
            double* gt = tree + 4 * n;
            gt[0] = gx; gt[1] = gy; gt[2] = g + vnorm2(nx - gx, ny - gy); gt[3] = slot;
            n++;
            status = 0;
            break;
        }
    }
    *n_nodes = n;
    if (draws) *draws = cur;
    return status;
}

/* OpenMP over independent queries (bench cpu_baseline): query q uses rnd + q * stride. */
int oracle_rrt_batch(int star, const double* rect, int nr, const double* circ, int nc, const double* bnd, int nb,
                     double delta, double X, double Y, const double* starts, const double* goals, int nq,
                     int sample_num, double max_dist, double radius, double goal_rate, const double* rnd,
                     int64_t stride, double* tree, int cap, int32_t* n_nodes, int32_t* status, int nthreads)
{
    if (nthreads <= 0) nthreads = omp_get_max_threads();
    int found = 0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) reduction(+ : found)
    for (int q = 0; q < nq; q++) {
        int nn = 0;
        status[q] = oracle_rrt(star, rect, nr, circ, nc, bnd, nb, delta, X, Y, starts[2 * q], starts[2 * q + 1],
                               goals[2 * q], goals[2 * q + 1], sample_num, max_dist, radius, goal_rate,
                               rnd + q * stride, stride, tree + (size_t)q * cap * 4, cap, &nn, NULL);
        n_nodes[q] = nn;
        found += status[q] == 0;
    }
    return found;
}

/* OpenMP over independent AStar3D queries with per-query occupancy occ [nq][X*Y*Z] (bench
 * cpu_baseline of config C5).  cost [nq]; status [nq]. */
int oracle_graph3d_batch(int algo, const uint8_t* occ, int X, int Y, int Z, int heuristic, const int32_t* s,
                         const int32_t* g, int nq, double* cost, int32_t* status, int nthreads)
{
    if (nthreads <= 0) nthreads = omp_get_max_threads();
    const int64_t ncell = (int64_t)X * Y * Z;
    int found = 0;
#pragma omp parallel num_threads(nthreads) reduction(+ : found)
    {
        int32_t* path = (int32_t*)malloc(sizeof(int32_t) * (size_t)(ncell + 1));
        int32_t plen, nexp;
        int64_t ctr[4];
#pragma omp for schedule(dynamic, 4)
        for (int q = 0; q < nq; q++) {
            status[q] = oracle_graph3d(algo, occ + (size_t)q * ncell, X, Y, Z, heuristic, s + 3 * q, g + 3 * q, cost + q, path,
                                       (int)(ncell + 1), &plen, NULL, 0, &nexp, ctr);
            found += status[q] == 0;
        }
        free(path);
    }
    return found;
}

int oracle_astar3d_batch(const uint8_t* occ, int X, int Y, int Z, int heuristic, const int32_t* s,
                         const int32_t* g, int nq, double* cost, int32_t* status, int nthreads)
{
    return oracle_graph3d_batch(0, occ, X, Y, Z, heuristic, s, g, nq, cost, status, nthreads);
}

/* ------------------------------------------------------------------------------------ */
/* LPAStar.plan (global_planner/graph_search/lpa_star.py:78-87): computeShortestPath      */
/* (:139-160) + extractPath (:209-230).  U is the reference's Python list, restated as   */
/* a list: `min(U, key=key)` = first minimal element in list order, `U.remove` shifts    */
/* the tail left, `heapq.heappush` appends and sifts by LNode.__lt__ (key list compare,  */
/* :32-33) on whatever order the list holds.                                           */
/* ------------------------------------------------------------------------------------ */
typedef struct {
    int32_t* cell;
    double *k1, *k2;
    int64_t n;
} ulist_t;

static inline int key_lt(double a1, double a2, double b1, double b2) { return a1 < b1 || (a1 == b1 && a2 < b2); }

static void u_remove(ulist_t* U, int32_t* pos, int64_t i)
{
    for (int64_t j = i; j + 1 < U->n; j++) {
        U->cell[j] = U->cell[j + 1];
        U->k1[j] = U->k1[j + 1];
        U->k2[j] = U->k2[j + 1];
        pos[U->cell[j]] = (int32_t)j;
    }
    U->n--;
}

static void u_push(ulist_t* U, int32_t* pos, int32_t c, double k1, double k2)
{
    int64_t p = U->n++;
    while (p > 0) { /* Lib/heapq.py _siftdown */
        int64_t q = (p - 1) >> 1;
        if (!key_lt(k1, k2, U->k1[q], U->k2[q])) break;
        U->cell[p] = U->cell[q];
        U->k1[p] = U->k1[q];
        U->k2[p] = U->k2[q];
        pos[U->cell[p]] = (int32_t)p;
        p = q;
    }
    U->cell[p] = c;
    U->k1[p] = k1;
    U->k2[p] = k2;
    pos[c] = (int32_t)p;
}

/* GraphSearcher.h of the LPA* key (:181-194): euclidean hypot or manhattan */
static inline double lpa_h(int heuristic, int x, int y, int gx, int gy)
{
    return heuristic == 1 ? (double)(abs(gx - x) + abs(gy - y)) : vnorm2((double)(gx - x), (double)(gy - y));
}

/* updateVertex (:162-179).  Returns 4 when the reference raises (KeyError off the map, or min()
 * of an empty neighbour list). */
static int lpa_update(const uint8_t* occ, int W, int H, int heuristic, int32_t src, int gx, int gy, double km,
                      double* g, double* rhs, int32_t* pos, ulist_t* U, int32_t v, int64_t* npush)
{
    const int x = v / H, y = v % H;
    if (v != src) {
        double best = INFINITY;
        int any = 0;
        for (int m = 0; m < 8; m++) { /* getNeighbor (:196-207): map lookup, then the obstacle filter */
            const int ux = x + MX8[m], uy = y + MY8[m];
            if (ux < 0 || uy < 0 || ux >= W || uy >= H) return 4;
            if (occ[(int64_t)ux * H + uy]) continue;
            const double c = collide2(occ, W, H, ux, uy, x, y) ? INFINITY : ((m & 1) ? sqrt(2.0) : 1.0);
            const double val = g[ux * H + uy] + c;
            if (!any || val < best) best = val;
            any = 1;
        }
        if (!any) return 4;
        rhs[v] = best;
    }
    if (pos[v] >= 0) {
        const int64_t i = pos[v];
        pos[v] = -1;
        u_remove(U, pos, i);
    }
    if (g[v] != rhs[v]) {
        const double mn = g[v] < rhs[v] ? g[v] : rhs[v];
        u_push(U, pos, v, mn + lpa_h(heuristic, x, y, gx, gy) + km, mn);
        (*npush)++;
    }
    return 0;
}

/* one greedy step of extractPath / D* Lite's OnPress walk: first minimal-g neighbour in motion order
 * among the free ones isCollision allows; -1 where the reference raises */
static int lpa_greedy(const uint8_t* occ, int W, int H, const double* g, int32_t c)
{
    const int x = c / H, y = c % H;
    int bm = -1;
    double bg = 0.0;
    for (int m = 0; m < 8; m++) {
        const int ux = x + MX8[m], uy = y + MY8[m];
        if (ux < 0 || uy < 0 || ux >= W || uy >= H) return -1;
        if (occ[(int64_t)ux * H + uy] || collide2(occ, W, H, x, y, ux, uy)) continue;
        if (bm < 0 || g[ux * H + uy] < bg) { bm = m; bg = g[ux * H + uy]; }
    }
    return bm;
}

/* status 0 found, 1 extractPath gave up after 1000 steps (cost kept, path empty), 4 the reference
 * raises (U empties: min() of an empty list; or KeyError / empty neighbour list).
 * path: start -> goal.  counters: {pushes, expansions (len(EXPAND)), path steps, max |U|}.
 * lite = 1: DStarLite.plan (d_star_lite.py:14-187, plan() inherited from LPAStar): the search runs
 * from the goal (rhs = 0) toward the start, keys add h(node, start) + km (km = 0 in plan()), a popped
 * node with an outdated key is re-keyed (:104-106), updateVertex skips the goal (:131-132), and
 * extractPath walks from the start to the goal without reversing (:156-187). */
static int lpa_core(int lite, const uint8_t* occ_in, int W, int H, int heuristic, int sx, int sy, int gx, int gy,
                    double* cost_out, int32_t* path, int path_cap, int32_t* path_len, int64_t* counters,
                    const int32_t* toggles, int nt, double* rp_cost, int32_t* rp_nexp, int32_t* rp_status)
{
    const int64_t ncell = (int64_t)W * H;
    uint8_t* occ = (uint8_t*)malloc((size_t)ncell); /* OnPress edits the obstacle set */
    memcpy(occ, occ_in, (size_t)ncell);
    double* g = (double*)malloc(sizeof(double) * (size_t)ncell);
    double* rhs = (double*)malloc(sizeof(double) * (size_t)ncell);
    int32_t* pos = (int32_t*)malloc(sizeof(int32_t) * (size_t)ncell);
    ulist_t U = {(int32_t*)malloc(sizeof(int32_t) * (size_t)ncell), (double*)malloc(sizeof(double) * (size_t)ncell),
                 (double*)malloc(sizeof(double) * (size_t)ncell), 0};
    int64_t npush = 0, nexp = 0, maxn = 0, steps = 0;
    int status = 0;
    *cost_out = 0.0;
    *path_len = 0;
    for (int64_t i = 0; i < ncell; i++) { g[i] = INFINITY; rhs[i] = INFINITY; pos[i] = -1; }
    const int32_t start = sx * H + sy, goal = gx * H + gy;
    /* src: the node created with rhs = 0; tgt: the node whose consistency ends the search and
     * toward which h points */
    const int32_t src = lite ? goal : start, tgt = lite ? start : goal;
    const int tx = lite ? sx : gx, ty = lite ? sy : gy, ox = lite ? gx : sx, oy = lite ? gy : sy;
    if (lite && start == goal) {
        /* map[start] overwrote map[goal] (:58-59): the goal node in U is detached, its g = 0 never
         * reaches a neighbour's rhs, so the first expansion pushes nothing and U empties */
        free(g); free(rhs); free(pos); free(U.cell); free(U.k1); free(U.k2); free(occ);
        if (counters) { counters[0] = 1; counters[1] = 1; counters[2] = 0; counters[3] = 1; }
        return 4;
    }
    rhs[src] = 0.0; /* LNode(start, inf, 0.0, None) (lpa_star.py:59); LNode(goal, inf, 0.0) (d_star_lite.py:57) */
    u_push(&U, pos, src, lpa_h(heuristic, ox, oy, tx, ty), 0.0);
    npush++;
    maxn = 1;
    /* phase 0: plan(); phase p >= 1: OnPress at toggles[p - 1] -- LPAStar's (lpa_star.py:101-137):
     * edit, then plan(); DStarLite's (d_star_lite.py:61-97): walk from the start along min-g
     * neighbours, after the first step set km = h(step, start), edit, computeShortestPath, walk on */
    double km = 0.0, wcost = 0.0;
    int32_t wcur = tgt;
    int64_t wlen = 0;
    for (int phase = 0; phase <= nt; phase++) {
    int walk_only = 0;
    if (phase > 0) {
        nexp = 0;
        steps = 0;
        *cost_out = 0.0;
        *path_len = 0;
        if (lite) {
            wcur = tgt;
            wcost = 0.0;
            wlen = 0;
            if (wlen < path_cap) path[wlen] = wcur;
            wlen++;
            if (wcur == src) {
                walk_only = 1;
            } else {
                const int bm = lpa_greedy(occ, W, H, g, wcur);
                if (bm < 0) status = 4;
                else {
                    const int x = wcur / H, y = wcur % H;
                    wcost += (bm & 1) ? sqrt(2.0) : 1.0;
                    wcur = (x + MX8[bm]) * H + (y + MY8[bm]);
                    if (wlen < path_cap) path[wlen] = wcur;
                    wlen++;
                    steps++;
                    km = lpa_h(heuristic, x + MX8[bm], y + MY8[bm], sx, sy);
                }
            }
        }
    }
    if (phase > 0 && !walk_only && !status) {
        const int cx = toggles[2 * phase - 2], cy = toggles[2 * phase - 1];
        const int32_t cc = cx * H + cy;
        if (!occ[cc]) {
            occ[cc] = 1;
        } else {
            occ[cc] = 0;
            status = lpa_update(occ, W, H, heuristic, src, tx, ty, km, g, rhs, pos, &U, cc, &npush);
        }
        for (int m = 0; m < 8 && !status; m++) { /* getNeighbor(node_change) raises before any update */
            const int ux = cx + MX8[m], uy = cy + MY8[m];
            if (ux < 0 || uy < 0 || ux >= W || uy >= H) status = 4;
        }
        for (int m = 0; m < 8 && !status; m++) {
            const int ux = cx + MX8[m], uy = cy + MY8[m];
            if (occ[(int64_t)ux * H + uy]) continue;
            status = lpa_update(occ, W, H, heuristic, src, tx, ty, km, g, rhs, pos, &U, ux * H + uy, &npush);
        }
    }
    for (;;) {
        if (status || walk_only) break;
        if (U.n == 0) { status = 4; break; }
        int64_t bi = 0;
        for (int64_t i = 1; i < U.n; i++)
            if (key_lt(U.k1[i], U.k2[i], U.k1[bi], U.k2[bi])) bi = i;
        /* start == goal: self.goal is a separate LNode(goal, inf, inf) that map[] no longer holds
         * (map[start] overwrote it, :62-63), so its g = rhs = inf forever and the loop only ends
         * when U empties */
        const double gg = start == goal ? INFINITY : g[tgt], grhs = start == goal ? INFINITY : rhs[tgt];
        const double gm = gg < grhs ? gg : grhs;
        const double gk1 = gm + 0.0 + km; /* calculateKey(tgt): h(tgt, tgt) = 0 */
        if (!key_lt(U.k1[bi], U.k2[bi], gk1, gm) && grhs == gg) break;
        const int32_t v = U.cell[bi];
        const double vk1 = U.k1[bi], vk2 = U.k2[bi];
        pos[v] = -1;
        u_remove(&U, pos, bi);
        nexp++;
        const int x = v / H, y = v % H;
        if (lite) { /* node.key < calculateKey(node): re-key, push, nothing else (:104-106) */
            const double mn = g[v] < rhs[v] ? g[v] : rhs[v];
            const double c1 = mn + lpa_h(heuristic, x, y, tx, ty) + km, c2 = mn;
            if (key_lt(vk1, vk2, c1, c2)) {
                u_push(&U, pos, v, c1, c2);
                npush++;
                if (U.n > maxn) maxn = U.n;
                continue;
            }
        }
        if (g[v] > rhs[v]) {
            g[v] = rhs[v];
        } else {
            g[v] = INFINITY;
            if ((status = lpa_update(occ, W, H, heuristic, src, tx, ty, km, g, rhs, pos, &U, v, &npush))) break;
        }
        for (int m = 0; m < 8 && !status; m++) {
            const int ux = x + MX8[m], uy = y + MY8[m];
            if (ux < 0 || uy < 0 || ux >= W || uy >= H) { status = 4; break; }
            if (occ[(int64_t)ux * H + uy]) continue;
            status = lpa_update(occ, W, H, heuristic, src, tx, ty, km, g, rhs, pos, &U, ux * H + uy, &npush);
        }
        if (status) break;
        if (U.n > maxn) maxn = U.n;
    }
    if (status == 0 && lite && phase > 0) { /* the rest of OnPress's walk: no step limit (a bound here) */
        while (wcur != src) {
            const int bm = lpa_greedy(occ, W, H, g, wcur);
            if (bm < 0) { status = 4; break; }
            const int x = wcur / H, y = wcur % H;
            wcost += (bm & 1) ? sqrt(2.0) : 1.0;
            wcur = (x + MX8[bm]) * H + (y + MY8[bm]);
            if (wlen < path_cap) path[wlen] = wcur;
            wlen++;
            if (++steps > 4 * ncell + 4) { status = 3; break; }
        }
        *cost_out = wcost;
        if (status == 0) {
            if (wlen > path_cap) status = 2;
            *path_len = (int32_t)wlen;
        }
    } else if (status == 0) { /* extractPath: greedy min-g neighbour from tgt, first minimum in motion order */
        int32_t c = tgt;
        double cost = 0.0;
        int64_t len = 0;
        if (len < path_cap) path[len] = c;
        len++;
        while (c != src) {
            const int x = c / H, y = c % H;
            int bm = -1;
            double bg = 0.0;
            for (int m = 0; m < 8; m++) {
                const int ux = x + MX8[m], uy = y + MY8[m];
                if (ux < 0 || uy < 0 || ux >= W || uy >= H) { status = 4; break; }
                if (occ[(int64_t)ux * H + uy] || collide2(occ, W, H, x, y, ux, uy)) continue;
                if (bm < 0 || g[ux * H + uy] < bg) { bm = m; bg = g[ux * H + uy]; }
            }
            if (status) break;
            if (bm < 0) { status = 4; break; }
            cost += (bm & 1) ? sqrt(2.0) : 1.0;
            c = (x + MX8[bm]) * H + (y + MY8[bm]);
            if (len < path_cap) path[len] = c;
            len++;
            if (++steps == 1000) { status = 1; break; }
        }
        *cost_out = cost;
        if (status == 0) {
            if (len > path_cap) status = 2;
            else if (!lite) /* LPA*: list(reversed(path)); D* Lite's path already runs start -> goal */
                for (int64_t i = 0; i < len / 2; i++) { int32_t t = path[i]; path[i] = path[len - 1 - i]; path[len - 1 - i] = t; }
            *path_len = (int32_t)len;
        }
    }
    if (nt > 0) {
        rp_cost[phase] = (status == 0 || status == 1) ? *cost_out : 0.0;
        rp_nexp[phase] = (int32_t)nexp;
        rp_status[phase] = status;
    }
    if (status != 0 && status != 1) {
        for (int p2 = phase + 1; p2 <= nt; p2++) { rp_cost[p2] = 0.0; rp_nexp[p2] = 0; rp_status[p2] = -1; }
        break;
    }
    if (status == 1 && phase < nt) status = 0;
    } /* phase */
    if (counters) { counters[0] = npush; counters[1] = nexp; counters[2] = steps; counters[3] = maxn; }
    free(g); free(rhs); free(pos); free(U.cell); free(U.k1); free(U.k2); free(occ);
    return status;
}

int oracle_lpastar2d(const uint8_t* occ, int W, int H, int heuristic, int sx, int sy, int gx, int gy,
                     double* cost_out, int32_t* path, int path_cap, int32_t* path_len, int64_t* counters)
{
    return lpa_core(0, occ, W, H, heuristic, sx, sy, gx, gy, cost_out, path, path_cap, path_len, counters, NULL, 0,
                    NULL, NULL, NULL);
}

/* LPAStar.plan() followed by nt OnPress edits (lpa_star.py:101-137) at toggles[nt][2]: rp_* [nt + 1]
 * hold each plan's cost / len(EXPAND) / status (-1 = not run: an earlier plan raised); path is the
 * last plan's. */
int oracle_lpastar2d_replan(int lite, const uint8_t* occ, int W, int H, int heuristic, int sx, int sy, int gx, int gy,
                            const int32_t* toggles, int nt, double* rp_cost, int32_t* rp_nexp, int32_t* rp_status,
                            int32_t* path, int path_cap, int32_t* path_len, int64_t* counters)
{
    double c;
    return lpa_core(lite, occ, W, H, heuristic, sx, sy, gx, gy, &c, path, path_cap, path_len, counters, toggles, nt,
                    rp_cost, rp_nexp, rp_status);
}

int oracle_dstarlite2d(const uint8_t* occ, int W, int H, int heuristic, int sx, int sy, int gx, int gy,
                       double* cost_out, int32_t* path, int path_cap, int32_t* path_len, int64_t* counters)
{
    return lpa_core(1, occ, W, H, heuristic, sx, sy, gx, gy, cost_out, path, path_cap, path_len, counters, NULL, 0,
                    NULL, NULL, NULL);
}

/* OpenMP batch of the LPAStar / DStarLite restatement (one grid, many queries; the bench's CPU
 * baseline).  Outputs per query: cost, status, n_expanded. */
void oracle_lpastar2d_batch(int lite, const uint8_t* occ, int W, int H, int heuristic, const int32_t* starts,
                            const int32_t* goals, int nq, double* cost, int32_t* status, int32_t* n_expanded,
                            int nthreads)
{
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4)
    for (int q = 0; q < nq; q++) {
        int32_t path[1002], plen;
        int64_t ctr[4];
        status[q] = lpa_core(lite, occ, W, H, heuristic, starts[2 * q], starts[2 * q + 1], goals[2 * q], goals[2 * q + 1],
                             &cost[q], path, 1002, &plen, ctr, NULL, 0, NULL, NULL, NULL);
        n_expanded[q] = (int32_t)ctr[1];
    }
}

/* OpenMP batch of the replanning restatement (plan() + nt OnPress edits per session, one toggle
 * list of nt cells per query): the bench's CPU baseline.  rp_* [nq][nt + 1] as in
 * oracle_lpastar2d_replan. */
void oracle_lpastar2d_replan_batch(int lite, const uint8_t* occ, int W, int H, int heuristic, const int32_t* starts,
                                   const int32_t* goals, int nq, const int32_t* toggles, int nt, double* rp_cost,
                                   int32_t* rp_nexp, int32_t* rp_status, int nthreads)
{
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4)
    for (int q = 0; q < nq; q++) {
        int32_t path[1002], plen;
        int64_t ctr[4];
        double c;
        const size_t o = (size_t)q * (size_t)(nt + 1);
        lpa_core(lite, occ, W, H, heuristic, starts[2 * q], starts[2 * q + 1], goals[2 * q], goals[2 * q + 1], &c, path,
                 1002, &plen, ctr, toggles + (size_t)q * 2 * (size_t)nt, nt, rp_cost + o, rp_nexp + o, rp_status + o);
    }
}

/* OpenMP batch of the DStar restatement (one grid, many queries; the bench's CPU baseline):
 * cost, status, n_process per query. */
void oracle_dstar2d_batch(const uint8_t* occ, int W, int H, const int32_t* starts, const int32_t* goals, int nq,
                          double* cost, int32_t* status, int64_t* n_process, int nthreads)
{
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
    {
        int32_t* path = (int32_t*)malloc(sizeof(int32_t) * ((size_t)W * H + 1));
#pragma omp for schedule(dynamic, 1)
        for (int q = 0; q < nq; q++) {
            int32_t plen;
            status[q] = oracle_dstar2d(occ, W, H, starts[2 * q], starts[2 * q + 1], goals[2 * q], goals[2 * q + 1],
                                       &cost[q], path, W * H + 1, &plen, &n_process[q], 0);
        }
        free(path);
    }
}

/* ============================================================================================
 * DStar3D (global_planner/graph_search/d_star3d.py:60-281): plan() (:100-109) followed by
 * nrounds apply_dynamic_obstacles() calls (:115-149).  OPEN is restated as the reference's Python
 * list: append only when the node is not in it (:245-246; Node3D equality is by coordinates and
 * "in OPEN" <=> t == OPEN throughout), min_state = the FIRST minimal k in list order (:220-225),
 * delete = list.remove (:248-253).  getNeighbor (:266-280) keeps in-map voxels with
 * isCollision(node, n) false; isCollision (graph_search_3d.py:66-107) is asymmetric for three-axis
 * diagonals.  `p in self.obstacles` is false outside the grid (only in-grid voxels are tested).
 * start == goal: map[start] = self.start detaches the goal object (:89-90): slot ncell.
 * ============================================================================================ */
typedef struct {
    double *h, *k;
    int32_t* parent;
    uint8_t* t;
    int32_t* open;
    int64_t nopen, capopen;
    uint8_t* occ; /* working copy (apply_dynamic_obstacles adds voxels) */
    int X, Y, Z, ncell, goal_slot, goal_cell;
    int64_t np;
} d3_t;

static inline int d3_occ(const d3_t* S, int x, int y, int z)
{
    if (x < 0 || y < 0 || z < 0 || x >= S->X || y >= S->Y || z >= S->Z) return 0;
    return S->occ[((int64_t)x * S->Y + y) * S->Z + z] != 0;
}
static inline void d3_xyz(const d3_t* S, int c, int* x, int* y, int* z)
{
    *z = c % S->Z;
    *y = (c / S->Z) % S->Y;
    *x = c / (S->Z * S->Y);
}
static inline int d3_coord(const d3_t* S, int slot) { return slot == S->goal_slot ? S->goal_cell : slot; }
/* isCollision(node1, node2) on voxel ids */
static int d3_coll(const d3_t* S, int a, int b)
{
    int x1, y1, z1, x2, y2, z2;
    d3_xyz(S, a, &x1, &y1, &z1);
    d3_xyz(S, b, &x2, &y2, &z2);
    if (d3_occ(S, x1, y1, z1) || d3_occ(S, x2, y2, z2)) return 1;
    const int dx = x2 - x1, dy = y2 - y1, dz = z2 - z1;
    const int ax = abs(dx) > abs(dy) ? abs(dx) : abs(dy);
    if ((ax > abs(dz) ? ax : abs(dz)) > 1) return 0;
    const int ch = (dx != 0) + (dy != 0) + (dz != 0);
    if (ch <= 1) return 0;
    if (ch == 2) {
        if (dx != 0 && dy != 0) return d3_occ(S, x1 + dx, y1, z1) || d3_occ(S, x1, y1 + dy, z1);
        if (dx != 0 && dz != 0) return d3_occ(S, x1 + dx, y1, z1) || d3_occ(S, x1, y1, z1 + dz);
        return d3_occ(S, x1, y1 + dy, z1) || d3_occ(S, x1, y1, z1 + dz);
    }
    return d3_occ(S, x1 + dx, y1, z1) || d3_occ(S, x1, y1 + dy, z1) || d3_occ(S, x1, y1, z1 + dz);
}
/* GraphSearcher3D.cost: inf on collision, else Planner3D.dist (math.sqrt of the squared deltas) */
static double d3_cost(const d3_t* S, int a, int b)
{
    if (d3_coll(S, a, b)) return INFINITY;
    int x1, y1, z1, x2, y2, z2;
    d3_xyz(S, a, &x1, &y1, &z1);
    d3_xyz(S, b, &x2, &y2, &z2);
    const double dx = x2 - x1, dy = y2 - y1, dz = z2 - z1;
    return sqrt(dx * dx + dy * dy + dz * dz);
}
/* insert (:233-246) */
static void d3_insert(d3_t* S, int slot, double h_new)
{
    if (S->t[slot] == T_NEW) S->k[slot] = h_new;
    else if (S->t[slot] == T_OPEN) S->k[slot] = S->k[slot] < h_new ? S->k[slot] : h_new;
    else if (S->t[slot] == T_CLOSED) S->k[slot] = S->h[slot] < h_new ? S->h[slot] : h_new;
    const int in_open = S->t[slot] == T_OPEN;
    S->h[slot] = h_new;
    S->t[slot] = T_OPEN;
    if (!in_open) {
        if (S->nopen == S->capopen) {
            S->capopen *= 2;
            S->open = (int32_t*)realloc(S->open, sizeof(int32_t) * (size_t)S->capopen);
        }
        S->open[S->nopen++] = slot;
    }
}
/* min_state (:220-225): first minimal k; returns the list index or -1 */
static int64_t d3_min_state(const d3_t* S)
{
    if (S->nopen == 0) return -1;
    int64_t bi = 0;
    for (int64_t i = 1; i < S->nopen; i++)
        if (S->k[S->open[i]] < S->k[S->open[bi]]) bi = i;
    return bi;
}
/* the neighbours of slot X (getNeighbor :266-280) as voxel ids, in motion order */
static int d3_neighbors(const d3_t* S, int Xs, int* nb)
{
    const int c = d3_coord(S, Xs);
    int x, y, z, n = 0;
    d3_xyz(S, c, &x, &y, &z);
    for (int m = 0; m < 26; m++) {
        const int nx = x + M3[m][0], ny = y + M3[m][1], nz = z + M3[m][2];
        if (nx < 0 || ny < 0 || nz < 0 || nx >= S->X || ny >= S->Y || nz >= S->Z) continue;
        const int v = (nx * S->Y + ny) * S->Z + nz;
        if (!d3_coll(S, c, v)) nb[n++] = v;
    }
    return n;
}
/* processState (:168-218); returns the new min k or -1 */
static double d3_process(d3_t* S)
{
    const int64_t mi = d3_min_state(S);
    if (mi < 0) return -1.0;
    const int Xs = S->open[mi];
    S->np++;
    const double k_old = S->k[Xs];
    /* delete (:248-253) */
    if (S->t[Xs] == T_OPEN) S->t[Xs] = T_CLOSED;
    memmove(S->open + mi, S->open + mi + 1, sizeof(int32_t) * (size_t)(S->nopen - mi - 1));
    S->nopen--;
    const int Xc = d3_coord(S, Xs);
    int nb[26];
    const int nn = d3_neighbors(S, Xs, nb);
    if (k_old < S->h[Xs])
        for (int i = 0; i < nn; i++) {
            const int n = nb[i];
            const double c = d3_cost(S, Xc, n);
            if (S->h[n] <= k_old && S->h[Xs] > S->h[n] + c) {
                S->parent[Xs] = n;
                S->h[Xs] = S->h[n] + c;
            }
        }
    if (k_old == S->h[Xs]) {
        for (int i = 0; i < nn; i++) {
            const int n = nb[i];
            const double c = d3_cost(S, Xc, n);
            if (S->t[n] == T_NEW || (S->parent[n] == Xc && S->h[n] != S->h[Xs] + c) ||
                (S->parent[n] != Xc && S->h[n] > S->h[Xs] + c)) {
                S->parent[n] = Xc;
                d3_insert(S, n, S->h[Xs] + c);
            }
        }
    } else {
        for (int i = 0; i < nn; i++) {
            const int n = nb[i];
            const double c = d3_cost(S, Xc, n);
            if (S->t[n] == T_NEW || (S->parent[n] == Xc && S->h[n] != S->h[Xs] + c)) {
                S->parent[n] = Xc;
                d3_insert(S, n, S->h[Xs] + c);
            } else if (S->parent[n] != Xc && S->h[n] > S->h[Xs] + c) {
                d3_insert(S, Xs, S->h[Xs]);
            } else if (S->parent[n] != Xc && S->h[Xs] > S->h[n] + c && S->t[n] == T_CLOSED && S->h[n] > k_old) {
                d3_insert(S, n, S->h[n]);
            }
        }
    }
    const int64_t s = d3_min_state(S);
    return s >= 0 ? S->k[S->open[s]] : -1.0;
}
/* modify (:255-264) */
static void d3_modify(d3_t* S, int node, double h_new, int64_t max_process)
{
    if (S->t[node] == T_CLOSED) d3_insert(S, node, h_new);
    for (;;) {
        const double k_min = d3_process(S);
        if (k_min < 0 || k_min >= S->h[node]) break;
        if (max_process > 0 && S->np >= max_process) break;
    }
}

/* Returns 0, or 3 when a cap was hit.  Per round r (0 = plan): cost[r], status[r] (0 reached the
 * goal, 1 stopped at a node without parent, 3 step / processState cap), nproc[r] = len(EXPAND),
 * path[r * path_cap ..] (voxel ids, start -> goal) and plen[r]. */
int oracle_dstar3d(const uint8_t* occ_in, int X, int Y, int Z, const int32_t* s, const int32_t* g,
                   const int32_t* blocks, int nrounds, int nblk, double* cost, int32_t* status, int64_t* nproc,
                   int32_t* path, int path_cap, int32_t* plen, int64_t max_process)
{
    d3_t S;
    S.X = X; S.Y = Y; S.Z = Z;
    S.ncell = X * Y * Z;
    const int start = (s[0] * Y + s[1]) * Z + s[2];
    S.goal_cell = (g[0] * Y + g[1]) * Z + g[2];
    S.goal_slot = start == S.goal_cell ? S.ncell : S.goal_cell;
    const int ns = S.ncell + 1;
    S.h = (double*)malloc(sizeof(double) * ns);
    S.k = (double*)malloc(sizeof(double) * ns);
    S.parent = (int32_t*)malloc(sizeof(int32_t) * ns);
    S.t = (uint8_t*)malloc(ns);
    S.occ = (uint8_t*)malloc(S.ncell);
    memcpy(S.occ, occ_in, S.ncell);
    S.capopen = 1024;
    S.nopen = 0;
    S.open = (int32_t*)malloc(sizeof(int32_t) * S.capopen);
    S.np = 0;
    for (int i = 0; i < ns; i++) {
        S.h[i] = INFINITY; S.k[i] = INFINITY; S.parent[i] = -1; S.t[i] = T_NEW;
    }
    S.h[S.goal_slot] = 0.0;
    d3_insert(&S, S.goal_slot, 0.0);
    int rc = 0;
    /* plan (:100-109) */
    for (;;) {
        const double kmin = d3_process(&S);
        if (kmin < 0) break;
        if (S.t[start] == T_CLOSED) break;
        if (max_process > 0 && S.np >= max_process) { rc = 3; break; }
    }
    const int64_t bound = 4 * (int64_t)S.ncell + 4;
    for (int r = 0; r <= nrounds; r++) {
        int32_t* pth = path + (size_t)r * path_cap;
        int n = 0, st = 0;
        double c = 0.0;
        if (r > 0) {
            const int32_t* b = blocks + ((size_t)(r - 1) * nblk) * 3;
            for (int i = 0; i < nblk; i++)
                if (b[3 * i] >= 0 && b[3 * i] < X && b[3 * i + 1] >= 0 && b[3 * i + 1] < Y && b[3 * i + 2] >= 0 &&
                    b[3 * i + 2] < Z)
                    S.occ[((int64_t)b[3 * i] * Y + b[3 * i + 1]) * Z + b[3 * i + 2]] = 1;
            S.np = 0;
        }
        int node = start;
        int64_t steps = 0;
        if (rc == 0) {
            if (r == 0) { if (n < path_cap) pth[n] = start; n++; }
            while (node != S.goal_cell) {
                if (++steps > bound) { st = 3; break; }
                if (S.parent[node] < 0) {
                    if (r > 0) d3_modify(&S, node, S.h[S.goal_slot] + d3_cost(&S, node, S.goal_cell), max_process);
                    st = 1;
                    break;
                }
                const int p = S.parent[node];
                const int pslot = p == S.goal_cell ? S.goal_slot : p;
                if (r > 0 && d3_coll(&S, node, p)) {
                    d3_modify(&S, node, S.h[pslot] + d3_cost(&S, node, p), max_process);
                    if (max_process > 0 && S.np >= max_process) { st = 3; break; }
                    continue;
                }
                if (r > 0) { if (n < path_cap) pth[n] = node; n++; }
                c += d3_cost(&S, node, p);
                node = p;
                if (r == 0) { if (n < path_cap) pth[n] = node; n++; }
            }
            if (r > 0 && st == 0 && node == S.goal_cell) { if (n < path_cap) pth[n] = node; n++; }
        } else {
            st = 3;
        }
        if (st == 3) rc = 3;
        cost[r] = c;
        status[r] = st;
        nproc[r] = S.np;
        plen[r] = n;
    }
    free(S.h); free(S.k); free(S.parent); free(S.t); free(S.open); free(S.occ);
    return rc;
}

/* ============================================================================================
 * DStar.plan (d_star.py:75-89) followed by npress OnPress(event) calls (:102-134) without the
 * figure.  processState (:158-218) with the list-semantics OPEN of oracle_dstar2d; OnPress adds the
 * obstacle (a free in-grid cell only), resets EXPAND, walks from the start along the parents
 * (path without the goal) and calls modify (:262-274) where an edge collides.
 * Per call r (0 = plan): cost[r], plen[r], path[r * path_cap ..], nproc[r] = len(EXPAND) (a None
 * appended by processState on an empty OPEN counts), status[r]: 0 done, 1 the press did nothing,
 * 2 path_cap overflow, 3 a loop the reference never leaves (4*W*H+4 walk steps, or modify on an
 * empty OPEN) or max_process, 4 the reference raises, -1 not run.
 * ============================================================================================ */
/* returns 0 = OPEN empty on entry (-1), 1 = processed, OPEN non-empty, 2 = processed, OPEN empty
 * (min_k raises), 3 = allocation failure, 4 = getNeighbor raised KeyError (*raise_cell = the node) */
static int d2_process(dstate_t* S, const uint8_t* occ, int W, int H, int64_t* np, int32_t* raise_cell)
{
    int64_t pos = d_minpos(S);
    (*np)++;
    if (pos < 0) return 0;
    int32_t x = S->open[pos];
    double k_old = S->k[x];
    if (S->t[x] == T_OPEN) S->t[x] = T_CLOSED;
    memmove(&S->open[pos], &S->open[pos + 1], sizeof(int32_t) * (size_t)(S->nopen - pos - 1));
    S->nopen--;
    const int32_t xc = x == S->goal_slot ? S->goal_cell : x; /* node.current */
    /* getNeighbor (:276-291): self.map[node + motion] for all 8 motions before the collision test;
     * self.map holds the in-grid cells only (env.py:34-35): a border node raises KeyError */
    if (xc / H == 0 || xc % H == 0 || xc / H == W - 1 || xc % H == H - 1) { *raise_cell = xc; return 4; }
    int32_t nb[8];
    double nc[8];
    int nn = d_neighbors(occ, W, H, xc, nb, nc);
    if (k_old < S->h[x])
        for (int i = 0; i < nn; i++) {
            int32_t y = nb[i];
            if (S->h[y] <= k_old && S->h[x] > S->h[y] + nc[i]) { S->parent[x] = y; S->h[x] = S->h[y] + nc[i]; }
        }
    if (k_old == S->h[x]) {
        for (int i = 0; i < nn; i++) {
            int32_t y = nb[i];
            if (S->t[y] == T_NEW || (S->parent[y] == xc && S->h[y] != S->h[x] + nc[i]) ||
                (S->parent[y] != xc && S->h[y] > S->h[x] + nc[i])) {
                S->parent[y] = xc;
                if (d_insert(S, y, S->h[x] + nc[i])) return 3;
            }
        }
    } else {
        for (int i = 0; i < nn; i++) {
            int32_t y = nb[i];
            if (S->t[y] == T_NEW || (S->parent[y] == xc && S->h[y] != S->h[x] + nc[i])) {
                S->parent[y] = xc;
                if (d_insert(S, y, S->h[x] + nc[i])) return 3;
            } else if (S->parent[y] != xc && S->h[y] > S->h[x] + nc[i]) {
                if (d_insert(S, x, S->h[x])) return 3;
            } else if (S->parent[y] != xc && S->h[x] > S->h[y] + nc[i] && S->t[y] == T_CLOSED && S->h[y] > k_old) {
                if (d_insert(S, y, S->h[y])) return 3;
            }
        }
    }
    return S->nopen == 0 ? 2 : 1;
}

int oracle_dstar2d_onpress(const uint8_t* occ_in, int W, int H, int sx, int sy, int gx, int gy, const int32_t* presses,
                           int npress, double* cost, int32_t* path, int path_cap, int32_t* plen, int64_t* nproc,
                           int32_t* status, int64_t max_process)
{
    const int64_t ncell = (int64_t)W * H;
    uint8_t* occ = (uint8_t*)malloc((size_t)ncell);
    memcpy(occ, occ_in, (size_t)ncell);
    dstate_t S;
    const int64_t ns = ncell + 1;
    S.h = (double*)malloc(sizeof(double) * (size_t)ns);
    S.k = (double*)malloc(sizeof(double) * (size_t)ns);
    S.parent = (int32_t*)malloc(sizeof(int32_t) * (size_t)ns);
    S.t = (uint8_t*)malloc((size_t)ns);
    S.capopen = 1024;
    S.nopen = 0;
    S.open = (int32_t*)malloc(sizeof(int32_t) * (size_t)S.capopen);
    for (int64_t i = 0; i < ns; i++) { S.h[i] = INFINITY; S.k[i] = INFINITY; S.parent[i] = -1; S.t[i] = T_NEW; }
    const int32_t start = sx * H + sy, goal = gx * H + gy;
    S.goal_cell = goal;
    S.goal_slot = start == goal ? (int32_t)ncell : goal;
    S.h[S.goal_slot] = 0.0; /* DNode(goal, None, 'NEW', 0, inf) (:58) */
    d_insert(&S, S.goal_slot, 0.0);
    int64_t np = 0;
    int st = 0;
    int32_t raise_cell = -1;
    int plen0 = 0; /* round 0's path length when it raises: -2 = getNeighbor's KeyError (path[0] = the node) */
    for (;;) {
        const int ps = d2_process(&S, occ, W, H, &np, &raise_cell);
        if (ps == 3) { st = 3; break; }
        if (ps == 4) { st = 4; plen0 = -2; break; }
        if (ps != 1) { st = 4; break; }
        if (S.t[start] == T_CLOSED) break;
        if (max_process > 0 && np >= max_process) { st = 3; break; }
    }
    for (int r = 0; r <= npress; r++) {
        int32_t* pth = path + (size_t)r * path_cap;
        int n = 0, rst = st;
        double c = 0.0;
        if (r == 0) {
            if (plen0 == -2) { n = -2; pth[0] = raise_cell; }
            if (st == 0) {
                int32_t x = start;
                pth[n++] = x;
                while (x != goal) {
                    int32_t p = S.parent[x];
                    if (p < 0 || n > ncell) { rst = 4; break; }
                    const int cx = x / H, cy = x % H, px = p / H, py = p % H;
                    c += collide2(occ, W, H, cx, cy, px, py) ? INFINITY : ((cx != px && cy != py) ? sqrt(2.0) : 1.0);
                    x = p;
                    if (n < path_cap) pth[n] = x;
                    n++;
                }
                if (rst == 0 && n > path_cap) rst = 2;
            }
        } else if (st != 0) {
            rst = -1;
        } else {
            const int px = presses[2 * (r - 1)], py = presses[2 * (r - 1) + 1];
            if (px < 0 || px > W - 1 || py < 0 || py > H - 1 || occ[(int64_t)px * H + py]) {
                rst = 1;
            } else {
                occ[(int64_t)px * H + py] = 1;
                np = 0;
                int32_t node = start;
                int64_t steps = 0;
                while (node != goal) {
                    if (++steps > 4 * ncell + 4) { rst = 3; break; }
                    const int32_t p = S.parent[node];
                    if (p < 0) { rst = 4; n = -1; break; } /* self.map[None]: KeyError */
                    const int cx = node / H, cy = node % H, qx = p / H, qy = p % H;
                    if (collide2(occ, W, H, cx, cy, qx, qy)) {
                        if (S.t[node] == T_CLOSED && d_insert(&S, node, S.h[p] + INFINITY)) { rst = 3; break; }
                        for (;;) {
                            const int ps = d2_process(&S, occ, W, H, &np, &raise_cell);
                            if (ps == 3) { rst = 3; break; }
                            if (ps == 4) { rst = 4; n = -2; pth[0] = raise_cell; break; }
                            if (ps == 2) { rst = 4; break; }
                            if (ps == 0) { rst = 3; break; } /* -1 >= node.h never holds: endless loop */
                            if (max_process > 0 && np >= max_process) { rst = 3; break; }
                            if (S.k[S.open[d_minpos(&S)]] >= S.h[node]) break;
                        }
                        if (rst != 0) break;
                        continue;
                    }
                    if (n < path_cap) pth[n] = node;
                    n++;
                    c += (cx != qx && cy != qy) ? sqrt(2.0) : 1.0;
                    node = p;
                }
                if (rst == 0 && n > path_cap) rst = 2;
            }
            if (rst == 3 || rst == 4) st = rst;
        }
        cost[r] = c;
        plen[r] = n;
        status[r] = rst;
        nproc[r] = rst == -1 ? 0 : np;
    }
    free(occ); free(S.h); free(S.k); free(S.parent); free(S.t); free(S.open);
    return st;
}

/* ============================================================================================
 * LPAStar3D (global_planner/graph_search/lpa_star3d.py:40-225): plan() (:78-82) = computeShortest
 * Path (:127-145) + extractPath (:185-225), and apply_change(coord, blocked) (:93-124) rounds.
 * U is restated as the reference's Python list: min(U, key) = the first minimal key (list `<`,
 * :130), U.remove = first occurrence (coordinate equality; the list never holds a node twice),
 * heapq.heappush = append + CPython _siftdown under LNode3D.__lt__ (key list compare, :38-40) on
 * whatever order the list has.  getNeighbor (:160-182): in the map and the endpoint not an
 * obstacle (no edge test); updateVertex's cost(n, node) uses isCollision(n, node) (asymmetric).
 * start == goal: map[goal] overwrites map[start] (:62-63), so the start object lives in slot ncell.
 * ============================================================================================ */
typedef struct {
    int32_t c;
    double k1, k2;
} l3ent_t;

typedef struct {
    double *g, *rhs;
    l3ent_t* U;
    int64_t n, cap;
    d3_t geo; /* X, Y, Z, ncell, occ, goal_slot (unused), goal_cell */
    int start_slot, start_cell, goal;
    int heur;
    int64_t nexp;
} l3_t;

static inline int l3_lt(const l3ent_t* a, const l3ent_t* b) { return a->k1 < b->k1 || (a->k1 == b->k1 && a->k2 < b->k2); }
static inline int l3_coord(const l3_t* S, int slot) { return slot == S->start_slot ? S->start_cell : slot; }
static double l3_h(const l3_t* S, int c)
{
    int x, y, z, gx, gy, gz;
    d3_xyz(&S->geo, c, &x, &y, &z);
    d3_xyz(&S->geo, S->goal, &gx, &gy, &gz);
    const int dx = abs(gx - x), dy = abs(gy - y), dz = abs(gz - z);
    if (S->heur == 1) return (double)(dx + dy + dz);
    return sqrt((double)(dx * dx + dy * dy + dz * dz));
}
/* getNeighbor (:160-182): slots of the in-map, non-obstacle neighbours of voxel c, motion order */
static int l3_neighbors(const l3_t* S, int c, int* nb)
{
    int x, y, z, k = 0;
    d3_xyz(&S->geo, c, &x, &y, &z);
    for (int m = 0; m < 26; m++) {
        const int nx = x + M3[m][0], ny = y + M3[m][1], nz = z + M3[m][2];
        if (nx < 0 || ny < 0 || nz < 0 || nx >= S->geo.X || ny >= S->geo.Y || nz >= S->geo.Z) continue;
        if (d3_occ(&S->geo, nx, ny, nz)) continue;
        nb[k++] = (nx * S->geo.Y + ny) * S->geo.Z + nz;
    }
    return k;
}
static void l3_push(l3_t* S, int32_t c, double k1, double k2)
{
    if (S->n == S->cap) {
        S->cap *= 2;
        S->U = (l3ent_t*)realloc(S->U, sizeof(l3ent_t) * (size_t)S->cap);
    }
    l3ent_t it = {c, k1, k2};
    int64_t pos = S->n++;
    while (pos > 0) { /* heapq._siftdown(heap, 0, pos) */
        const int64_t parent = (pos - 1) >> 1;
        if (l3_lt(&it, &S->U[parent])) {
            S->U[pos] = S->U[parent];
            pos = parent;
            continue;
        }
        break;
    }
    S->U[pos] = it;
}
static void l3_remove_at(l3_t* S, int64_t i)
{
    memmove(S->U + i, S->U + i + 1, sizeof(l3ent_t) * (size_t)(S->n - i - 1));
    S->n--;
}
static int64_t l3_find(const l3_t* S, int32_t slot)
{
    for (int64_t i = 0; i < S->n; i++)
        if (l3_coord(S, S->U[i].c) == l3_coord(S, slot)) return i; /* Node3D equality: coordinates */
    return -1;
}
/* updateVertex (:147-158) */
static void l3_update(l3_t* S, int32_t slot)
{
    const int c = l3_coord(S, slot);
    if (c != S->start_cell) { /* node != self.start: coordinate equality */
        int nb[26];
        const int k = l3_neighbors(S, c, nb);
        if (k) {
            double best = INFINITY;
            for (int i = 0; i < k; i++) {
                const double v = S->g[nb[i]] + d3_cost(&S->geo, nb[i], c);
                if (i == 0 || v < best) best = v;
            }
            S->rhs[slot] = best;
        } else {
            S->rhs[slot] = INFINITY;
        }
    }
    const int64_t p = l3_find(S, slot);
    if (p >= 0) l3_remove_at(S, p);
    if (S->g[slot] != S->rhs[slot]) {
        const double m = S->g[slot] < S->rhs[slot] ? S->g[slot] : S->rhs[slot];
        l3_push(S, slot, m + l3_h(S, c), m);
    }
}
/* computeShortestPath (:127-145) */
static int l3_compute(l3_t* S, int64_t max_exp)
{
    while (S->n > 0) {
        int64_t bi = 0;
        for (int64_t i = 1; i < S->n; i++)
            if (l3_lt(&S->U[i], &S->U[bi])) bi = i;
        const int gs = S->goal;
        const double gm = S->g[gs] < S->rhs[gs] ? S->g[gs] : S->rhs[gs];
        const l3ent_t gk = {0, gm + l3_h(S, S->goal), gm};
        if (!l3_lt(&S->U[bi], &gk) && S->rhs[gs] == S->g[gs]) break;
        const int32_t v = S->U[bi].c;
        l3_remove_at(S, bi);
        S->nexp++;
        if (max_exp > 0 && S->nexp > max_exp) return 3;
        if (S->g[v] > S->rhs[v]) {
            S->g[v] = S->rhs[v];
        } else {
            S->g[v] = INFINITY;
            l3_update(S, v);
        }
        int nb[26];
        const int k = l3_neighbors(S, l3_coord(S, v), nb);
        for (int i = 0; i < k; i++) l3_update(S, nb[i]);
    }
    return 0;
}
/* extractPath (:185-225): greedy min-g neighbours from the goal; (cost, []) when stuck or after
 * 100000 steps.  Returns the path length written (start -> goal) or -1 for an empty path. */
static int64_t l3_extract(const l3_t* S, double* cost, int32_t* path, int64_t path_cap)
{
    int node = S->goal;
    double c = 0.0;
    int64_t n = 0, safety = 0;
    int32_t* tmp = (int32_t*)malloc(sizeof(int32_t) * 100002);
    tmp[n++] = node;
    while (node != S->start_cell) {
        int nb[26], cand[26], k = l3_neighbors(S, node, nb), nc = 0;
        for (int i = 0; i < k; i++)
            if (!d3_coll(&S->geo, node, nb[i])) cand[nc++] = nb[i];
        if (!nc) { *cost = c; free(tmp); return -1; }
        int best = cand[0];
        for (int i = 1; i < nc; i++)
            if (S->g[cand[i]] < S->g[best]) best = cand[i];
        c += d3_cost(&S->geo, node, best);
        node = best;
        tmp[n++] = node;
        if (++safety >= 100000) { *cost = c; free(tmp); return -1; }
    }
    *cost = c;
    for (int64_t i = 0; i < n && i < path_cap; i++) path[i] = tmp[n - 1 - i];
    free(tmp);
    return n;
}

/* changes [nr][4] = (x, y, z, mode): mode 0 toggle (blocked=None), 1 block, 2 free.  Per call r
 * (0 = plan): cost[r], plen[r] (0 = the reference's empty path), path[r * path_cap ..],
 * nexp[r] = len(EXPAND), status[r]: 0 path, 1 empty path, 2 path_cap overflow, 3 cap. */
int oracle_lpastar3d(const uint8_t* occ_in, int X, int Y, int Z, int heuristic, const int32_t* s, const int32_t* g,
                     const int32_t* changes, int nr, double* cost, int32_t* status, int64_t* nexp, int32_t* path,
                     int path_cap, int32_t* plen, int64_t max_exp)
{
    l3_t S;
    S.geo.X = X; S.geo.Y = Y; S.geo.Z = Z;
    S.geo.ncell = X * Y * Z;
    S.geo.occ = (uint8_t*)malloc(S.geo.ncell);
    memcpy(S.geo.occ, occ_in, S.geo.ncell);
    S.heur = heuristic;
    S.start_cell = (s[0] * Y + s[1]) * Z + s[2];
    S.goal = (g[0] * Y + g[1]) * Z + g[2];
    S.start_slot = S.start_cell == S.goal ? S.geo.ncell : S.start_cell;
    S.geo.goal_slot = -1;
    S.geo.goal_cell = -1;
    const int ns = S.geo.ncell + 1;
    S.g = (double*)malloc(sizeof(double) * ns);
    S.rhs = (double*)malloc(sizeof(double) * ns);
    for (int i = 0; i < ns; i++) { S.g[i] = INFINITY; S.rhs[i] = INFINITY; }
    S.rhs[S.start_slot] = 0.0; /* LNode3D(start, inf, 0.0) */
    S.cap = 1024;
    S.n = 0;
    S.U = (l3ent_t*)malloc(sizeof(l3ent_t) * (size_t)S.cap);
    l3_push(&S, S.start_slot, 0.0 + l3_h(&S, S.start_cell), 0.0); /* calculateKey(start) */
    int rc = 0;
    for (int r = 0; r <= nr; r++) {
        S.nexp = 0; /* EXPAND.clear() in apply_change; empty at construction */
        int st = 0;
        if (r > 0) {
            const int32_t* ch = changes + (size_t)(r - 1) * 4;
            const int cx = ch[0], cy = ch[1], cz = ch[2], mode = ch[3];
            const int in = cx >= 0 && cy >= 0 && cz >= 0 && cx < X && cy < Y && cz < Z;
            const int cell = in ? (cx * Y + cy) * Z + cz : -1;
            const int is_obs = in && S.geo.occ[cell];
            if (in) {
                if (mode == 0) {
                    if (is_obs) { S.geo.occ[cell] = 0; l3_update(&S, cell); }
                    else S.geo.occ[cell] = 1;
                } else if (mode == 1) {
                    S.geo.occ[cell] = 1;
                } else if (is_obs) {
                    S.geo.occ[cell] = 0;
                    l3_update(&S, cell);
                }
                int nb[26];
                const int k = l3_neighbors(&S, cell, nb);
                for (int i = 0; i < k; i++) l3_update(&S, nb[i]);
            }
        }
        if (l3_compute(&S, max_exp)) st = 3;
        double c = 0.0;
        int64_t n = 0;
        if (st == 0) {
            n = l3_extract(&S, &c, path + (size_t)r * path_cap, path_cap);
            if (n < 0) { st = 1; n = 0; }
            else if (n > path_cap) st = 2;
        }
        cost[r] = c;
        status[r] = st;
        nexp[r] = S.nexp;
        plen[r] = (int32_t)n;
        if (st == 3) { rc = 3; for (int q = r + 1; q <= nr; q++) status[q] = -1; break; }
    }
    free(S.geo.occ); free(S.g); free(S.rhs); free(S.U);
    return rc;
}

/* OpenMP batches of the DStar3D / LPAStar3D restatements over per-query grids occ[nq][X*Y*Z]
 * (plan + nr rounds of changes; the bench's CPU baselines): per query and call cost, status,
 * len(EXPAND) at [q * (nr + 1) + r]. */
void oracle_dstar3d_batch(const uint8_t* occ, int per_query, int X, int Y, int Z, const int32_t* s, const int32_t* g,
                          int nq, const int32_t* blocks, int nr, int nblk, double* cost, int32_t* status, int64_t* nproc,
                          int nthreads)
{
    if (nthreads > 0) omp_set_num_threads(nthreads);
    const size_t nc = (size_t)X * Y * Z;
#pragma omp parallel
    {
        int32_t* path = (int32_t*)malloc(sizeof(int32_t) * (nc + 1) * (size_t)(nr + 1));
        int32_t* plen = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nr + 1));
#pragma omp for schedule(dynamic, 4)
        for (int q = 0; q < nq; q++)
            oracle_dstar3d(occ + (per_query ? (size_t)q * nc : 0), X, Y, Z, s + 3 * q, g + 3 * q,
                           blocks ? blocks + (size_t)q * nr * nblk * 3 : NULL, nr, nblk, cost + (size_t)q * (nr + 1),
                           status + (size_t)q * (nr + 1), nproc + (size_t)q * (nr + 1), path, (int)nc + 1, plen, 0);
        free(path);
        free(plen);
    }
}

void oracle_lpastar3d_batch(const uint8_t* occ, int per_query, int X, int Y, int Z, int heuristic, const int32_t* s,
                            const int32_t* g, int nq, const int32_t* changes, int nr, double* cost, int32_t* status,
                            int64_t* nexp, int nthreads)
{
    if (nthreads > 0) omp_set_num_threads(nthreads);
    const size_t nc = (size_t)X * Y * Z;
#pragma omp parallel
    {
        int32_t* path = (int32_t*)malloc(sizeof(int32_t) * (nc + 1) * (size_t)(nr + 1));
        int32_t* plen = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nr + 1));
#pragma omp for schedule(dynamic, 4)
        for (int q = 0; q < nq; q++)
            oracle_lpastar3d(occ + (per_query ? (size_t)q * nc : 0), X, Y, Z, heuristic, s + 3 * q, g + 3 * q,
                             changes ? changes + (size_t)q * nr * 4 : NULL, nr, cost + (size_t)q * (nr + 1),
                             status + (size_t)q * (nr + 1), nexp + (size_t)q * (nr + 1), path, (int)nc + 1, plen, 0);
        free(path);
        free(plen);
    }
}

/* ==================================================================================== */
/* TimeOptimalTrajectory3D (trajectory/time_optimal_trajectory.py:8-353,                 */
/* trajectory_base.py:245-261): scipy CubicSpline per axis, forward/backward velocity     */
/* integration, interp1d sampling, yaw / yaw rate.                                         */
/* ==================================================================================== */

typedef struct {
    double vmax[3], amax[3];  /* TrajectoryConstraints.max_velocity / max_acceleration */
    double tstep;             /* TrajectoryConstraints.min_time_step */
    double res;               /* path_resolution */
} totp_params_t;

/* scipy CubicSpline(x, y) with bc 'not-a-knot' (scipy/interpolate/_cubic.py CubicSpline.__init__,
   scipy 1.15): first derivatives s[] at the knots.  n == 2: both ends take the slope; n == 3: the
   parabola system solved by LU with partial pivoting (LAPACK dgesv); n >= 4: the tridiagonal system
   with the not-a-knot end rows, banded LU with partial pivoting (LAPACK dgbtf2: multipliers by the
   reciprocal pivot) and the column-oriented banded back substitution (dtbsv). */
static void cspline_slopes(const double* x, const double* y, int n, double* s, double* w /* 5n */)
{
    double* dx = w;
    double* sl = w + n;
    for (int i = 0; i + 1 < n; i++) {
        dx[i] = x[i + 1] - x[i];
        sl[i] = (y[i + 1] - y[i]) / dx[i];
    }
    if (n == 2) {
        s[0] = sl[0];
        s[1] = sl[0];
        return;
    }
    if (n == 3) {
        double A[3][3] = {{1.0, 1.0, 0.0}, {dx[1], 2.0 * (dx[0] + dx[1]), dx[0]}, {0.0, 1.0, 1.0}};
        double b[3] = {2.0 * sl[0], 3.0 * (dx[0] * sl[1] + dx[1] * sl[0]), 2.0 * sl[1]};
        for (int k = 0; k < 3; k++) {
            int p = k;
            for (int r = k + 1; r < 3; r++)
                if (fabs(A[r][k]) > fabs(A[p][k])) p = r;
            if (p != k) {
                for (int c = 0; c < 3; c++) { double t = A[k][c]; A[k][c] = A[p][c]; A[p][c] = t; }
                double t = b[k]; b[k] = b[p]; b[p] = t;
            }
            const double rinv = 1.0 / A[k][k];
            for (int r = k + 1; r < 3; r++) {
                const double m = A[r][k] * rinv;
                for (int c = k + 1; c < 3; c++) A[r][c] -= m * A[k][c];
                b[r] -= m * b[k];
            }
        }
        for (int k = 2; k >= 0; k--) {
            s[k] = b[k] / A[k][k];
            for (int r = 0; r < k; r++) b[r] -= s[k] * A[r][k];
        }
        return;
    }
    /* rows: L = sub-diagonal (col i-1), D = diagonal, U1 = col i+1, U2 = col i+2 (pivoting fill) */
    double* D = w + 2 * n;
    double* U1 = w + 3 * n;
    double* U2 = w + 4 * n;
    double Lk1;  /* the sub-diagonal entry of the row below the current pivot row */
    double* b = s;
    for (int i = 1; i + 1 < n; i++) {
        D[i] = 2.0 * (dx[i - 1] + dx[i]);
        U1[i] = dx[i - 1];
        U2[i] = 0.0;
        b[i] = 3.0 * (dx[i] * sl[i - 1] + dx[i - 1] * sl[i]);
    }
    {
        const double d = x[2] - x[0];
        D[0] = dx[1];
        U1[0] = d;
        U2[0] = 0.0;
        b[0] = ((dx[0] + 2.0 * d) * dx[1] * sl[0] + (dx[0] * dx[0]) * sl[1]) / d;
    }
    double Lnm1;
    {
        const double d = x[n - 1] - x[n - 3];
        D[n - 1] = dx[n - 3];
        Lnm1 = d;
        U1[n - 1] = 0.0;
        U2[n - 1] = 0.0;
        b[n - 1] = ((dx[n - 2] * dx[n - 2]) * sl[n - 3] + (2.0 * d + dx[n - 2]) * dx[n - 3] * sl[n - 2]) / d;
    }
    for (int k = 0; k + 1 < n; k++) {
        Lk1 = (k + 1 == n - 1) ? Lnm1 : dx[k + 1];  /* A[k+1][k] (A[-1, :-2] = dx[1:]) */
        if (fabs(Lk1) > fabs(D[k])) {  /* swap rows k and k+1 (columns k .. k+2) */
            const double t0 = D[k], t1 = U1[k], t2 = U2[k], tb = b[k];
            D[k] = Lk1; U1[k] = D[k + 1]; U2[k] = U1[k + 1]; b[k] = b[k + 1];
            Lk1 = t0; D[k + 1] = t1; U1[k + 1] = t2; b[k + 1] = tb;
        }
        const double m = Lk1 * (1.0 / D[k]);
        D[k + 1] -= m * U1[k];
        if (k + 2 < n) U1[k + 1] -= m * U2[k];
        b[k + 1] -= m * b[k];
    }
    for (int j = n - 1; j >= 0; j--) {
        if (b[j] != 0.0) {
            b[j] = b[j] / D[j];
            const double t = b[j];
            if (j >= 1) b[j - 1] -= t * U1[j - 1];
            if (j >= 2) b[j - 2] -= t * U2[j - 2];
        }
    }
}

/* PPoly evaluation (scipy/interpolate/_ppoly.pyx find_interval_ascending + evaluate_poly1 with
   dx = 0): interval i with x[i] <= v < x[i+1] (the last closed), then sum_k c[K-1-k] (v - x[i])^k
   with the power built by repeated products.  c: K coefficient rows of n-1 segments. */
static int pp_interval(const double* x, int n, double v)
{
    if (!(x[0] <= v && v <= x[n - 1])) return v < x[0] ? 0 : n - 2;
    if (v == x[n - 1]) return n - 2;
    int lo = 0, hi = n - 2;
    if (v < x[lo + 1]) hi = lo;
    while (lo < hi) {
        const int mid = (hi + lo) / 2;
        if (v < x[mid]) hi = mid;
        else if (v >= x[mid + 1]) lo = mid + 1;
        else { lo = mid; break; }
    }
    return lo;
}

/* position, first and second derivative of one axis at v: the CubicSpline and its derivative(1) /
   derivative(2) PPolys (coefficients [3c0, 2c1, c2] and [6c0, 2c1], PPoly.derivative's rising
   factorials) */
static void pp_eval3(const double* c /* [4][n-1] */, const double* x, int n, double v, double* p, double* d1, double* d2)
{
    const int i = pp_interval(x, n, v), m = n - 1;
    const double s = v - x[i];
    const double c0 = c[i], c1 = c[m + i], c2 = c[2 * m + i], c3 = c[3 * m + i];
    const double s2 = s * s, s3 = s2 * s;
    *p = ((c3 + c2 * s) + c1 * s2) + c0 * s3;
    *d1 = (c2 + (2.0 * c1) * s) + (3.0 * c0) * s2;
    *d2 = (2.0 * c1) + (6.0 * c0) * s;
}

typedef struct {
    int n;              /* waypoints */
    double L;           /* path_length */
    const double* arc;  /* arc lengths [n] */
    const double* c;    /* per axis [4][n-1] */
} totp_path_t;

/* _evaluate_path (time_optimal_trajectory.py:76-94): s clipped to [0, L] */
static void totp_eval(const totp_path_t* P, double s, double pos[3], double q1[3], double q2[3])
{
    if (s < 0.0) s = 0.0;
    if (s > P->L) s = P->L;
    for (int d = 0; d < 3; d++) pp_eval3(P->c + (size_t)d * 4 * (P->n - 1), P->arc, P->n, s, &pos[d], &q1[d], &q2[d]);
}

/* _compute_max_velocity (:96-118) */
static double totp_vmax(const totp_path_t* P, const totp_params_t* T, double s)
{
    double pos[3], q1[3], q2[3];
    totp_eval(P, s, pos, q1, q2);
    double best = 0.0;
    int any = 0;
    for (int d = 0; d < 3; d++)
        if (fabs(q1[d]) > 1e-10) {
            const double v = T->vmax[d] / fabs(q1[d]);
            if (!any || v < best) best = v;
            any = 1;
        }
    if (!any) {
        best = T->vmax[0];
        for (int d = 1; d < 3; d++) if (T->vmax[d] < best) best = T->vmax[d];
    }
    return best;
}

/* _compute_max_acceleration (:120-160), including the reference's sign handling for q' < 0 */
static void totp_amax(const totp_path_t* P, const totp_params_t* T, double s, double sd, double* smax, double* smin)
{
    double pos[3], q1[3], q2[3];
    totp_eval(P, s, pos, q1, q2);
    double hi = INFINITY, lo = -INFINITY;
    for (int d = 0; d < 3; d++)
        if (fabs(q1[d]) > 1e-10) {
            const double cen = q2[d] * sd * sd;
            const double a = T->amax[d];
            const double fw = (a - cen) / q1[d], bw = (-a - cen) / q1[d];
            if (q1[d] > 0) {
                if (fw < hi) hi = fw;
                if (bw > lo) lo = bw;
            } else {
                if (-bw < hi) hi = -bw;
                if (-fw > lo) lo = -fw;
            }
        }
    *smax = hi;
    *smin = lo;
}

static double py_min(double a, double b) { return b < a ? b : a; }
static double np_sq(double a) { return a * a; }

/* One TimeOptimalTrajectory3D(path, constraints, path_resolution).generate().  Profiles of
   n_samples = max(int(L / res), 100) entries go to s_values / s_dot / s_ddot / time (up to
   sample_cap), trajectory points (time, position[3], velocity[3], acceleration[3], yaw, yaw rate;
   NaN for None) to pts (up to point_cap rows of 12).  Returns 0, 2 (a cap was too small: the
   counts are still reported) or 4 (fewer than 2 waypoints: the reference raises ValueError). */
int oracle_totp3d(const double* path, int n, const totp_params_t* T, int sample_cap, double* s_values, double* s_dot,
                  double* s_ddot, double* time_prof, int* n_samples, int point_cap, double* pts, int* n_points,
                  double* total_time)
{
    *n_samples = 0;
    *n_points = 0;
    *total_time = 0.0;
    if (n < 2) return 4;
    double* arc = (double*)malloc(sizeof(double) * n);
    double* c = (double*)malloc(sizeof(double) * 12 * (n - 1));
    double* w = (double*)malloc(sizeof(double) * 5 * n);
    double* y = (double*)malloc(sizeof(double) * n);
    double* sl = (double*)malloc(sizeof(double) * n);
    /* _parameterize_path (:41-74): cumulative arc length, np.linalg.norm = sqrt(dot) */
    arc[0] = 0.0;
    for (int i = 1; i < n; i++) {
        const double a = path[3 * i] - path[3 * i - 3], b = path[3 * i + 1] - path[3 * i - 2], e = path[3 * i + 2] - path[3 * i - 1];
        arc[i] = arc[i - 1] + sqrt((a * a + b * b) + e * e);
    }
    const double L = arc[n - 1];
    for (int i = 0; i + 1 < n; i++)
        if (!(arc[i + 1] - arc[i] > 0.0)) {  /* scipy: `x` must be strictly increasing (ValueError) */
            free(arc); free(c); free(w); free(y); free(sl);
            return 4;
        }
    for (int d = 0; d < 3; d++) {
        for (int i = 0; i < n; i++) y[i] = path[3 * i + d];
        cspline_slopes(arc, y, n, sl, w);
        /* CubicHermiteSpline coefficients (scipy/interpolate/_cubic.py) */
        double* cd = c + (size_t)d * 4 * (n - 1);
        for (int i = 0; i + 1 < n; i++) {
            const double dx = arc[i + 1] - arc[i], slope = (y[i + 1] - y[i]) / dx;
            const double t = ((sl[i] + sl[i + 1]) - 2.0 * slope) / dx;
            cd[i] = t / dx;
            cd[(n - 1) + i] = (slope - sl[i]) / dx - t;
            cd[2 * (n - 1) + i] = sl[i];
            cd[3 * (n - 1) + i] = y[i];
        }
    }
    totp_path_t P = {n, L, arc, c};
    int ns = (int)(L / T->res);
    if (ns < 100) ns = 100;
    *n_samples = ns;
    double* sv = (double*)malloc(sizeof(double) * ns);
    double* sd = (double*)malloc(sizeof(double) * ns);
    double* sdd = (double*)malloc(sizeof(double) * ns);
    double* tp = (double*)malloc(sizeof(double) * ns);
    np_linspace(0.0, L, ns, sv);
    /* _forward_integration (:162-195) */
    sd[0] = 0.0;
    for (int i = 1; i < ns; i++) {
        const double ds = sv[i] - sv[i - 1], smid = (sv[i] + sv[i - 1]) / 2.0;
        const double vc = totp_vmax(&P, T, smid);
        double smax, smin;
        totp_amax(&P, T, sv[i - 1], sd[i - 1], &smax, &smin);
        if (smax > 0) {
            const double v2 = np_sq(sd[i - 1]) + 2.0 * smax * ds;
            sd[i] = py_min(sqrt(v2 > 0 ? v2 : 0.0), vc);
        } else {
            sd[i] = py_min(sd[i - 1], vc);
        }
    }
    /* _backward_integration (:197-226) */
    sd[ns - 1] = 0.0;
    for (int i = ns - 2; i >= 0; i--) {
        const double ds = sv[i + 1] - sv[i];
        double smax, smin;
        totp_amax(&P, T, sv[i + 1], sd[i + 1], &smax, &smin);
        if (smin < 0) {
            const double v2 = np_sq(sd[i + 1]) - 2.0 * smin * ds;
            sd[i] = py_min(sd[i], sqrt(v2 > 0 ? v2 : 0.0));
        }
    }
    /* _compute_velocity_profile (:228-258) */
    for (int i = 0; i < ns; i++) sdd[i] = 0.0;
    for (int i = 1; i + 1 < ns; i++) {
        const double ds = sv[i + 1] - sv[i - 1];
        if (ds > 0) sdd[i] = (np_sq(sd[i + 1]) - np_sq(sd[i - 1])) / (2.0 * ds);
    }
    tp[0] = 0.0;
    for (int i = 1; i < ns; i++) {
        const double ds = sv[i] - sv[i - 1], avg = (sd[i] + sd[i - 1]) / 2.0;
        const double dt = avg > 1e-10 ? ds / avg : ds / 0.1;
        tp[i] = tp[i - 1] + dt;
    }
    const double total = tp[ns - 1];
    *total_time = total;
    int rc = 0;
    if (ns <= sample_cap) {
        memcpy(s_values, sv, sizeof(double) * ns);
        memcpy(s_dot, sd, sizeof(double) * ns);
        memcpy(s_ddot, sdd, sizeof(double) * ns);
        memcpy(time_prof, tp, sizeof(double) * ns);
    } else {
        rc = 2;
    }
    /* generate (:260-302): t = 0, dt, ... <= total_time, then total_time if the last is short */
    int np_ = 0;
    double t = 0.0, last_t = -1.0;
    for (;;) {
        int last = 0;
        double tq;
        if (t <= total) {
            tq = t;
        } else if (np_ > 0 && last_t < total) {
            tq = total;
            last = 1;
        } else {
            break;
        }
        if (np_ < point_cap) {
            /* evaluate (:304-335): interp1d linear (searchsorted left, clipped to [1, n-1]) */
            const double tc = tq < 0 ? 0 : (tq > total ? total : tq);
            int hi = 0;
            {
                int lo_ = 0, hi_ = ns;
                while (lo_ < hi_) { const int mid = (lo_ + hi_) / 2; if (tp[mid] < tc) lo_ = mid + 1; else hi_ = mid; }
                hi = lo_;
            }
            if (hi < 1) hi = 1;
            if (hi > ns - 1) hi = ns - 1;
            const int lo = hi - 1;
            const double xl = tp[lo], xh = tp[hi], dxl = tc - xl;
            const double s = (sv[hi] - sv[lo]) / (xh - xl) * dxl + sv[lo];
            const double sdt = (sd[hi] - sd[lo]) / (xh - xl) * dxl + sd[lo];
            const double sddt = (sdd[hi] - sdd[lo]) / (xh - xl) * dxl + sdd[lo];
            double pos[3], q1[3], q2[3];
            totp_eval(&P, s, pos, q1, q2);
            double* o = pts + (size_t)np_ * 12;
            o[0] = tc;
            for (int d = 0; d < 3; d++) {
                o[1 + d] = pos[d];
                o[4 + d] = q1[d] * sdt;
                o[7 + d] = q2[d] * np_sq(sdt) + q1[d] * sddt;
            }
            /* compute_yaw_from_velocity (trajectory_base.py:245-261) */
            o[10] = sqrt(o[4] * o[4] + o[5] * o[5]) > 1e-6 ? atan2(o[5], o[4]) : NAN;
            o[11] = NAN;
            if (np_ > 0) {
                const double* pr = o - 12;
                const double dtp = o[0] - pr[0];
                if (dtp > 0 && !isnan(o[10]) && !isnan(pr[10])) {
                    double dy = o[10] - pr[10];
                    while (dy > PI_) dy -= 2.0 * PI_;
                    while (dy < -PI_) dy += 2.0 * PI_;
                    o[11] = dy / dtp;
                }
            }
        }
        np_++;
        last_t = tq;
        if (last) break;
        t += T->tstep;
    }
    *n_points = np_;
    if (np_ > point_cap) rc = 2;
    free(arc); free(c); free(w); free(y); free(sl); free(sv); free(sd); free(sdd); free(tp);
    return rc;
}

/* batch over paths (path_off: waypoint offsets, nq + 1) with OpenMP over queries; per-query caps */
int oracle_totp3d_batch(const double* path, const int64_t* path_off, int nq, const totp_params_t* T, int sample_cap,
                        double* s_values, double* s_dot, double* s_ddot, double* time_prof, int* n_samples, int point_cap,
                        double* pts, int* n_points, double* total_time, int* status, int nthreads)
{
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
    for (int q = 0; q < nq; q++) {
        const size_t so = (size_t)q * sample_cap;
        status[q] = oracle_totp3d(path + 3 * path_off[q], (int)(path_off[q + 1] - path_off[q]), T, sample_cap,
                                  s_values + so, s_dot + so, s_ddot + so, time_prof + so, &n_samples[q], point_cap,
                                  pts + (size_t)q * point_cap * 12, &n_points[q], &total_time[q]);
    }
    return 0;
}

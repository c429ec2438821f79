/*
 * bh_oracle.c — TEST INFRASTRUCTURE ONLY (tests/, bench.py cpu_baseline).
 *
 * CPU restatement of BarnesHutSystem::update (src/systems/barnes_hut.cpp:
 * 50-295, include/systems/barnes_hut.hpp:19-150): the sequential point-region
 * quadtree insertion and the recursive force walk, literally, over plain
 * arrays instead of the EnTT registry.  Pinned against the reference's own
 * barnes_hut.cpp compiled into oracle/_ref (ref_driver.cpp lpref_barnes_hut;
 * tests/test_oracle_bh.py, fixtures tests/golden/bh_*.npz).
 *
 * Bodies are the entities of view<Position, Mass>(exclude<Boundary>) in that
 * view's iteration order (the insertion order of buildTree, :117-128);
 * has_vel marks those that also have a Velocity (bodyView, :89).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "../include/lpe.h"

typedef struct {
    double totalMass, comX, comY;
    double bx, by, size;
    int isLeaf, allSmall;
    int single;                  /* body index, -1 = entt::null */
    int child;                   /* first of nw, ne, sw, se (-1: none) */
} Node;

typedef struct {
    Node *n;
    int count, cap;
    const double *x, *y, *m;
    double thr;
    int depth, maxDepth;
} Tree;

static int alloc_node(Tree *t) {                                   /* allocateNode :38-48 */
    if (t->count >= t->cap) {
        t->cap = t->cap ? 2 * t->cap : 1024;
        t->n = (Node *)realloc(t->n, sizeof(Node) * (size_t)t->cap);
    }
    Node *k = &t->n[t->count];
    memset(k, 0, sizeof(*k));
    k->isLeaf = 1;
    k->allSmall = 1;
    k->single = -1;
    k->child = -1;
    return t->count++;
}

static int contains(const Node *k, double x, double y) {            /* barnes_hut.hpp contains() */
    return x >= k->bx && x < k->bx + k->size && y >= k->by && y < k->by + k->size;
}

static int quadrant(const Node *k, double x, double y) {            /* barnes_hut.hpp getQuadrant() */
    double midX = k->bx + k->size * 0.5;
    double midY = k->by + k->size * 0.5;
    if (x < midX) return (y < midY) ? 0 : 2;
    return (y < midY) ? 1 : 3;
}

static void subdivide(Tree *t, int node) {                         /* :199-238 */
    int c = t->count;
    for (int i = 0; i < 4; i++) alloc_node(t);
    Node *k = &t->n[node];
    k->isLeaf = 0;
    double half = k->size * 0.5, x = k->bx, y = k->by;
    k->child = c;
    t->n[c + 0].bx = x;        t->n[c + 0].by = y;        t->n[c + 0].size = half;
    t->n[c + 1].bx = x + half; t->n[c + 1].by = y;        t->n[c + 1].size = half;
    t->n[c + 2].bx = x;        t->n[c + 2].by = y + half; t->n[c + 2].size = half;
    t->n[c + 3].bx = x + half; t->n[c + 3].by = y + half; t->n[c + 3].size = half;
}

static int insert(Tree *t, int node, int p, int level) {            /* insertParticle :133-197 */
    Node *k = &t->n[node];
    const double x = t->x[p], y = t->y[p], m = t->m[p];
    if (!contains(k, x, y)) return 0;
    if (level > t->maxDepth) return -1;                             /* safety cap (lpe.h) */
    if (level > t->depth) t->depth = level;
    if (k->totalMass == 0.0) {
        k->totalMass = m;
        k->comX = x;
        k->comY = y;
        k->single = p;
        if (m >= t->thr) k->allSmall = 0;
        return 0;
    }
    if (k->isLeaf) {
        int old = k->single;
        subdivide(t, node);
        if (insert(t, node, old, level) < 0) return -1;
        return insert(t, node, p, level);
    }
    double nt = k->totalMass + m;
    k->comX = (k->comX * k->totalMass + x * m) / nt;
    k->comY = (k->comY * k->totalMass + y * m) / nt;
    k->totalMass = nt;
    if (m >= t->thr) k->allSmall = 0;
    int c = k->child + quadrant(k, x, y);
    return insert(t, c, p, level + 1);
}

typedef struct {
    const lpe_bh_config *cfg;
    const Node *n;
    double dt;
} Walk;

static void force(const Walk *w, int node, int p, double px, double py, double pm,
                  double *vx, double *vy) {                         /* calculateForce :240-294 */
    const Node *k = &w->n[node];
    if (k->totalMass == 0.0) return;
    if (k->allSmall && w->cfg->small_mass_threshold > 0.0) return;
    double dx = k->comX - px;
    double dy = k->comY - py;
    double distSq = dx * dx + dy * dy + w->cfg->softener * w->cfg->softener;
    double dist = sqrt(distSq);
    double sizeSq = k->size * k->size;
    double thetaSq = w->cfg->theta * w->cfg->theta;
    int approx = k->isLeaf || (sizeSq / distSq < thetaSq);
    if (approx) {
        if (k->isLeaf && k->single == p) return;
        double f = w->cfg->G * k->totalMass * pm / distSq;
        double inv = f / (pm * dist);
        double ax = dx * inv;
        double ay = dy * inv;
        *vx += ax * w->dt;
        *vy += ay * w->dt;
    } else {
        for (int i = 0; i < 4; i++) force(w, k->child + i, p, px, py, pm, vx, vy);
    }
}

int lpeo_bh_config_default(lpe_bh_config *c) {
    c->theta = 0.5;
    c->small_mass_threshold = 1e3;
    c->universe_size = 0.0;
    c->softener = 0.0;
    c->G = 6.674e-11;
    return 0;
}

/* One BarnesHutSystem::update.  vx/vy are updated in place for the bodies
 * with has_vel (NULL: all).  Returns 0, or -1 when the tree exceeds
 * LPE_BH_MAX_DEPTH (a safety cap fp64 boxes never reach, lpe.h). */
int lpeo_bh_step(const lpe_bh_config *cfg, int n, const double *x, const double *y, double *vx,
                 double *vy, const double *m, const unsigned char *has_vel, double dt,
                 lpe_bh_stats *st) {
    if (st) memset(st, 0, sizeof(*st));
    if (cfg->small_mass_threshold > 0.0) {                          /* early exit :55-71 */
        int skip = 1;
        for (int i = 0; i < n; i++)
            if (m[i] >= cfg->small_mass_threshold) { skip = 0; break; }
        if (skip) {
            if (st) st->skipped = 1;
            return 0;
        }
    }
    Tree t;
    memset(&t, 0, sizeof(t));
    t.x = x; t.y = y; t.m = m;
    t.thr = cfg->small_mass_threshold;
    t.maxDepth = LPE_BH_MAX_DEPTH;
    int root = alloc_node(&t);                                      /* buildTree :101-131 */
    t.n[root].bx = 0.0;
    t.n[root].by = 0.0;
    t.n[root].size = cfg->universe_size;
    int ins = 0, rc = 0;
    for (int i = 0; i < n && rc == 0; i++) {
        if (x[i] >= 0.0 && x[i] < cfg->universe_size && y[i] >= 0.0 && y[i] < cfg->universe_size) {
            rc = insert(&t, root, i, 0);
            ins++;
        }
    }
    if (rc == 0) {
        Walk w = {cfg, t.n, dt};
        for (int i = 0; i < n; i++)                                 /* :89-98 */
            if (!has_vel || has_vel[i]) force(&w, root, i, x[i], y[i], m[i], &vx[i], &vy[i]);
    }
    if (st) {
        st->inserted = ins;
        st->nodes = t.count;
        st->depth = t.depth;
    }
    free(t.n);
    return rc;
}

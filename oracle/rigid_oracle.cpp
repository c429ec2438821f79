/*
 * rigid_oracle.cpp — TEST INFRASTRUCTURE ONLY.  CPU restatement of the
 * reference's rigid-body path (src/systems/rigid/ sources) and of the integrator
 * systems (src/systems/{gravity,rotation,movement,boundary,sleep}.cpp), used
 * as the parity checker for the HIP rigid path.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Parity status: PINNED against the reference itself.  oracle/_ref builds the
 * reference's own rigid sources (oracle/Makefile.ref) and tests/golden/
 * holds fixtures it produced (tests/golden/gen_rigid_golden.py); the stages
 * below reproduce them bit for bit given the same orders.  Exception:
 * contact_solver.cpp includes <arm_neon.h>, absent on x86-64, so the
 * reference PGS cannot be built here; lpeo_pgs restates it (the NEON use is a
 * 2-lane product + lane subtraction, contact_solver.cpp:207-214) and is
 * unpinned by reference execution.
 *
 * Orders.  The reference's pair order comes from its quadtree traversal and
 * its PGS order from std::unordered_map iteration (contact_manager.cpp:
 * 169-245), both platform/structure dependent; every stage here takes an
 * explicit order so fixtures recorded from the reference can be replayed, and
 * the canonical order (pairs sorted by entity id; solvers in the colour-major
 * order of lpeo_colour_order) is what the HIP path runs.
 * Arithmetic: IEEE double / float as in the reference, no FMA contraction
 * (build with -ffp-contract=off; g++ on x86-64 emits none by default).
 */
#include "rigid_oracle.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>
#include "../little-physics-engine_amd/csrc/lpe_trig.h"

/* Trigonometry of the restatement.  Portable (default): the implementation
 * the device shares (csrc/lpe_trig.h), so device and oracle agree bit for
 * bit.  libm (lpeo_set_libm_trig(1)): the platform's std::cos/std::sin, as
 * the reference calls them -- the mode the reference fixtures are checked
 * in (tests/test_oracle_rigid.py), bit for bit; the two modes differ only by
 * the libm's last-bit rounding (<= 1 ulp). */
static int g_libm_trig = 0;
extern "C" void lpeo_set_libm_trig(int on) { g_libm_trig = on != 0; }
static inline double ocos(double x) { return g_libm_trig ? std::cos(x) : lpe_cos(x); }
static inline double osin(double x) { return g_libm_trig ? std::sin(x) : lpe_sin(x); }
/* the fluid gather's std::cos(float) (fluid.cpp:399-400: rb.angle is a float) */
static inline float ocosf(float x) { return g_libm_trig ? std::cos(x) : lpe_cosf(x); }
static inline float osinf(float x) { return g_libm_trig ? std::sin(x) : lpe_sinf(x); }

namespace {

struct V2 {
    double x = 0, y = 0;
    V2() = default;
    V2(double a, double b) : x(a), y(b) {}
    V2 operator+(const V2 &o) const { return {x + o.x, y + o.y}; }
    V2 operator-(const V2 &o) const { return {x - o.x, y - o.y}; }
    V2 operator-() const { return {-x, -y}; }
    V2 operator*(double s) const { return {x * s, y * s}; }
    double dot(const V2 &o) const { return x * o.x + y * o.y; }       /* vector_math.cpp:118-120 */
    double cross(const V2 &o) const { return x * o.y - y * o.x; }     /* vector_math.cpp:122-124 */
    double length() const { return std::sqrt(x * x + y * y); }        /* vector_math.cpp:114-116 */
    V2 normalized() const {                                            /* vector_math.cpp:130-137 */
        double len = length();
        if (len > 1e-9) return {x / len, y / len};
        return {1.0, 0.0};
    }
};

/* ShapeData (polygon.hpp:113-119) */
struct Shape {
    bool circle;
    double radius;
    V2 pos;
    double angle;
    const double *lv;   /* local verts (x, y pairs) */
    int nv;
};

Shape shape_of(const lpe_body &b, const double *verts) {
    Shape s;
    s.circle = (b.flags & LPE_BODY_CIRCLE) != 0;        /* narrowphase.cpp:38-46 */
    s.radius = s.circle ? b.radius : 0.0;
    s.pos = V2(b.x, b.y);
    s.angle = (b.flags & LPE_BODY_HAS_ANGPOS) ? b.angle : 0.0;
    s.lv = verts + 2 * (size_t)b.vert_off;
    s.nv = s.circle ? 0 : b.vert_cnt;
    return s;
}

/* supportPolygon (polygon.hpp:55-76) */
V2 support_poly(const Shape &s, const V2 &d) {
    double c = ocos(s.angle), sn = osin(s.angle);
    double bestProj = -1e9;
    V2 best;
    for (int i = 0; i < s.nv; i++) {
        double lx = s.lv[2 * i], ly = s.lv[2 * i + 1];
        double wx = s.pos.x + (lx * c - ly * sn);
        double wy = s.pos.y + (lx * sn + ly * c);
        double proj = wx * d.x + wy * d.y;
        if (proj > bestProj) { bestProj = proj; best.x = wx; best.y = wy; }
    }
    return best;
}

/* supportCircle (polygon.hpp:90-101) */
V2 support_circle(const Shape &s, const V2 &d) {
    double len = std::sqrt(d.x * d.x + d.y * d.y);
    V2 dn = d;
    if (len > 1e-9) { dn.x /= len; dn.y /= len; }
    return V2(s.pos.x + dn.x * s.radius, s.pos.y + dn.y * s.radius);
}

/* supportMinkowski (polygon.hpp:132-141) */
V2 support(const Shape &A, const Shape &B, const V2 &d) {
    V2 pA = A.circle ? support_circle(A, d) : support_poly(A, d);
    V2 nd(-d.x, -d.y);
    V2 pB = B.circle ? support_circle(B, nd) : support_poly(B, nd);
    return V2(pA.x - pB.x, pA.y - pB.y);
}

/* handleSimplex (gjk.cpp:9-71); pts[0] is the oldest point */
bool handle_simplex(std::vector<V2> &pts, V2 &dir) {
    size_t count = pts.size();
    if (count == 2) {
        V2 a = pts[1], b = pts[0];
        V2 ab = b - a, ao = -a;
        if (ab.dot(ao) > 0) {
            V2 perp(-ab.y, ab.x);
            if (perp.dot(ao) < 0) perp = V2(ab.y, -ab.x);
            dir = perp;
        } else {
            pts = {a};
            dir = ao;
        }
        return false;
    }
    if (count == 3) {
        V2 a = pts[2], b = pts[1], c = pts[0];
        V2 ab = b - a, ac = c - a, ao = -a;
        V2 abPerp(ab.y, -ab.x);
        if (abPerp.dot(ac) > 0) abPerp = V2(-ab.y, ab.x);
        V2 acPerp(ac.y, -ac.x);
        if (acPerp.dot(ab) > 0) acPerp = V2(-ac.y, ac.x);
        if (ab.dot(ao) > 0 && abPerp.dot(ao) > 0) {
            pts.erase(pts.begin());
            dir = abPerp;
            return false;
        }
        if (ac.dot(ao) > 0 && acPerp.dot(ao) > 0) {
            pts.erase(pts.begin() + 1);
            dir = acPerp;
            return false;
        }
        return true;
    }
    dir = V2(1, 0);
    return false;
}

/* GJKIntersect (gjk.cpp:73-123) */
bool gjk(const Shape &A, const Shape &B, std::vector<V2> &pts) {
    V2 dir(1, 0);
    pts.clear();
    pts.push_back(support(A, B, dir));
    if (pts[0].dot(dir) < 0) return false;
    dir = -pts[0];
    int it = 0;
    while (true) {
        it++;
        if (it > 100) return false;
        V2 np = support(A, B, dir);
        double proj = np.dot(dir);
        if (proj < 0) return false;
        pts.push_back(np);
        if (handle_simplex(pts, dir)) return true;
    }
}

/* edgeDistance (epa.cpp:20-30) */
double edge_distance(const V2 &a, const V2 &b, V2 &normal) {
    V2 e = b - a;
    normal = V2(e.y, -e.x).normalized();
    double dist = normal.dot(a);
    if (dist < 0) { normal.x = -normal.x; normal.y = -normal.y; dist = -dist; }
    return dist;
}

/* EPA (epa.cpp:32-97) */
bool epa(const Shape &A, const Shape &B, const std::vector<V2> &simplex, V2 &n, double &pen) {
    std::vector<V2> poly = simplex;
    {
        V2 ab = poly[1] - poly[0], ac = poly[2] - poly[0];
        if (std::fabs(ab.cross(ac)) < 1e-14) return false;
    }
    {
        double cv = (poly[1].x - poly[0].x) * (poly[2].y - poly[0].y) -
                    (poly[1].y - poly[0].y) * (poly[2].x - poly[0].x);
        if (cv < 0) std::reverse(poly.begin(), poly.end());
    }
    for (int iter = 0; iter < 100; iter++) {
        double closest = std::numeric_limits<double>::max();
        int ce = -1;
        V2 en;
        for (int i = 0; i < (int)poly.size(); i++) {
            int j = (i + 1) % (int)poly.size();
            V2 nn;
            double d = edge_distance(poly[i], poly[j], nn);
            if (d < closest) { closest = d; ce = i; en = nn; }
        }
        if (ce < 0) return false;
        V2 p = support(A, B, en);
        double d = p.dot(en);
        if (d - closest < 1e-9) { n = en; pen = d; return true; }   /* EPSILON, vector_math.hpp:20 */
        poly.insert(poly.begin() + ((ce + 1) % (int)poly.size()), p);
    }
    return false;
}

/* getWorldVerts, polygon branch (narrowphase.cpp:56-81) */
std::vector<V2> world_verts(const Shape &s) {
    std::vector<V2> v;
    if (s.circle) {
        const int samples = 8;
        double step = (2.0 * M_PI) / samples;
        for (int i = 0; i < samples; i++) {
            double a = i * step + s.angle;
            v.emplace_back(s.pos.x + s.radius * ocos(a), s.pos.y + s.radius * osin(a));
        }
        return v;
    }
    for (int i = 0; i < s.nv; i++) {
        double lx = s.lv[2 * i], ly = s.lv[2 * i + 1];
        double rx = lx * ocos(s.angle) - ly * osin(s.angle);
        double ry = lx * osin(s.angle) + ly * ocos(s.angle);
        v.emplace_back(s.pos.x + rx, s.pos.y + ry);
    }
    return v;
}

/* findBestFace (narrowphase.cpp:126-145) */
int best_face(const std::vector<V2> &v, const V2 &normal) {
    int best = 0;
    double bestDot = -1e30;
    int n = (int)v.size();
    for (int i = 0; i < n; i++) {
        int j = (i + 1) % n;
        V2 e = v[j] - v[i];
        V2 fn = V2(-e.y, e.x).normalized();
        double d = fn.dot(normal);
        if (d > bestDot) { bestDot = d; best = i; }
    }
    return best;
}

/* clipFace (narrowphase.cpp:203-234) */
std::vector<V2> clip_face(const std::vector<V2> &poly, const V2 &pn, double off) {
    std::vector<V2> out;
    int n = (int)poly.size();
    for (int i = 0; i < n; i++) {
        int j = (i + 1) % n;
        const V2 &p1 = poly[i], &p2 = poly[j];
        double d1 = pn.dot(p1) - off, d2 = pn.dot(p2) - off;
        bool in1 = d1 <= 0.0, in2 = d2 <= 0.0;
        if (in1) out.push_back(p1);
        if (in1 != in2) {
            double t = d1 / (d1 - d2);
            out.push_back(p1 + (p2 - p1) * t);
        }
    }
    return out;
}

/* buildPolygonPolygonContacts (narrowphase.cpp:304-350) with the reference
 * face always on A (chooseReference, narrowphase.cpp:173-174). */
void poly_poly_contacts(const Shape &A, const Shape &B, const V2 &gn, int ia, int ib, int pair,
                        std::vector<lpe_contact> &out) {
    std::vector<V2> av = world_verts(A), bv = world_verts(B);
    int fa = best_face(av, gn);
    V2 ea = av[(fa + 1) % av.size()] - av[fa];
    V2 refN = V2(-ea.y, ea.x).normalized();
    /* clipIncidentPolygon (narrowphase.cpp:239-299) */
    V2 v1 = av[fa], v2 = av[(fa + 1) % av.size()];
    double faceOff = refN.dot(v1);
    V2 edge = (v2 - v1).normalized();
    V2 topN = edge;
    double topOff = topN.dot(v2);
    V2 botN = -edge;
    double botOff = botN.dot(v1);
    std::vector<V2> poly = bv;
    poly = clip_face(poly, refN, faceOff);
    poly = clip_face(poly, topN, topOff);
    poly = clip_face(poly, botN, botOff);
    double planeOff = refN.dot(v1);
    for (const V2 &cp : poly) {
        lpe_contact c{};
        c.a = ia; c.b = ib; c.pair = pair;
        c.nx = gn.x; c.ny = gn.y;
        c.pen = -(refN.dot(cp) - planeOff);
        c.px = cp.x; c.py = cp.y;
        out.push_back(c);
    }
}

bool is_solid(const lpe_body &b) { return (b.flags & LPE_BODY_SOLID) != 0; }

/* computeAABB (broadphase.cpp:158-191) */
void aabb(const lpe_body &b, const double *verts, double &mnx, double &mny, double &mxx,
          double &mxy) {
    double angle = (b.flags & LPE_BODY_HAS_ANGPOS) ? b.angle : 0.0;
    if (b.flags & LPE_BODY_CIRCLE) {
        double r = b.radius;
        mnx = b.x - r; mxx = b.x + r;
        mny = b.y - r; mxy = b.y + r;
        return;
    }
    mnx = b.x; mxx = b.x; mny = b.y; mxy = b.y;
    const double *lv = verts + 2 * (size_t)b.vert_off;
    for (int i = 0; i < b.vert_cnt; i++) {
        double vx = lv[2 * i], vy = lv[2 * i + 1];
        double rx = vx * ocos(angle) - vy * osin(angle);
        double ry = vx * osin(angle) + vy * ocos(angle);
        double wx = b.x + rx, wy = b.y + ry;
        if (wx < mnx) mnx = wx;
        if (wx > mxx) mxx = wx;
        if (wy < mny) mny = wy;
        if (wy > mxy) mxy = wy;
    }
}

}  // namespace

extern "C" void lpeo_rigid_config_default(lpe_rigid_config *c) {
    std::memset(c, 0, sizeof(*c));
    c->universeSize = 6.0;
    c->metersPerPixel = 0.01;
    c->quadtreeCapacity = 8;
    c->boundaryBuffer = 500.0;
    c->smallParticleThreshold = 0.01;
    c->pgsIterations = 10;
    c->frictionCoeff = 0.5f;
    c->posIterations = 10;
    c->baumgarte = 0.02;
    c->slop = 0.001;
    c->gravity = 9.8;
    c->planetaryMassThreshold = 1e10;
    c->angularDamping = 0.98;
    c->maxAngularSpeed = 20.0;
    c->marginPixels = 15.0;
    c->bounceDamping = 0.7;
    c->maxSpeed = 1.0;
    c->linearSleepThreshold = 0.5;
    c->angularSleepThreshold = 0.5;
    c->sleepFramesThreshold = 60;
}

extern "C" int lpeo_broadphase(const lpe_rigid_config *cfg, int nb, const lpe_body *bodies,
                               const double *verts, int32_t *pairs, int cap) {
    struct Box { int i; double mnx, mny, mxx, mxy; };
    std::vector<Box> boxes;
    const double lo = -cfg->boundaryBuffer;
    const double hi = -cfg->boundaryBuffer + (cfg->universeSize + 2 * cfg->boundaryBuffer);
    /* candidates: view<Position, Mass, ParticlePhase> with phase Solid
     * (broadphase.cpp:208-221, :250-257); only boxes overlapping the quadtree
     * root are inserted / find anything (BoxNode::insert/query, :92, :126-127) */
    for (int i = 0; i < nb; i++) {
        const lpe_body &b = bodies[i];
        if (!(b.flags & LPE_BODY_HAS_MASS) || !(b.flags & LPE_BODY_HAS_PHASE) || !is_solid(b)) continue;
        Box bx{i, 0, 0, 0, 0};
        aabb(b, verts, bx.mnx, bx.mny, bx.mxx, bx.mxy);
        if (bx.mxx < lo || bx.mnx > hi || bx.mxy < lo || bx.mny > hi) continue;
        boxes.push_back(bx);
    }
    std::sort(boxes.begin(), boxes.end(), [](const Box &a, const Box &b) {
        return a.mnx < b.mnx || (a.mnx == b.mnx && a.i < b.i);
    });
    std::vector<std::pair<uint64_t, std::pair<int, int>>> out;
    for (size_t p = 0; p < boxes.size(); p++) {
        const Box &A = boxes[p];
        for (size_t q = p + 1; q < boxes.size() && boxes[q].mnx <= A.mxx; q++) {
            const Box &B = boxes[q];
            if (A.mxy < B.mny || A.mny > B.mxy) continue;  /* boxesOverlap (:35-39) */
            const lpe_body &ba = bodies[A.i], &bb = bodies[B.i];
            if (ba.eid == bb.eid) continue;
            bool bothB = (ba.flags & LPE_BODY_BOUNDARY) && (bb.flags & LPE_BODY_BOUNDARY);
            double sa = std::max(A.mxx - A.mnx, A.mxy - A.mny);
            double sb = std::max(B.mxx - B.mnx, B.mxy - B.mny);
            bool bothSmall = sa < cfg->smallParticleThreshold && sb < cfg->smallParticleThreshold;
            if (bothB || bothSmall) continue;
            int ia = A.i, ib = B.i;
            if (bodies[ia].eid > bodies[ib].eid) std::swap(ia, ib);  /* (e, f) with f > e (:264) */
            uint64_t key = ((uint64_t)bodies[ia].eid << 32) | bodies[ib].eid;
            out.push_back({key, {ia, ib}});
        }
    }
    std::sort(out.begin(), out.end(),
              [](const auto &a, const auto &b) { return a.first < b.first; });
    int np = (int)out.size();
    if (np > cap) return -np;
    for (int k = 0; k < np; k++) { pairs[2 * k] = out[k].second.first; pairs[2 * k + 1] = out[k].second.second; }
    return np;
}

extern "C" int lpeo_narrowphase(int nb, const lpe_body *bodies, const double *verts, int np,
                                const int32_t *pairs, lpe_contact *outc, int cap) {
    (void)nb;
    std::vector<lpe_contact> out;
    std::vector<V2> simplex;
    for (int k = 0; k < np; k++) {
        int ia = pairs[2 * k], ib = pairs[2 * k + 1];
        Shape A = shape_of(bodies[ia], verts), B = shape_of(bodies[ib], verts);
        if (!gjk(A, B, simplex)) continue;
        V2 n;
        double pen;
        if (!epa(A, B, simplex, n, pen)) continue;
        lpe_contact c{};
        c.a = ia; c.b = ib; c.pair = k;
        c.nx = n.x; c.ny = n.y; c.pen = pen;
        if (A.circle && B.circle) {                  /* narrowphase.cpp:376-385 */
            V2 cp = B.pos - n * B.radius;
            c.px = cp.x; c.py = cp.y;
            out.push_back(c);
        } else if (A.circle && !B.circle) {          /* :386-395 */
            V2 cp = A.pos + n * A.radius;
            c.px = cp.x; c.py = cp.y;
            out.push_back(c);
        } else if (!A.circle && B.circle) {          /* :396-406 */
            V2 cp = B.pos - n * B.radius;
            c.px = cp.x; c.py = cp.y;
            out.push_back(c);
        } else {                                     /* :407-414 */
            poly_poly_contacts(A, B, n, ia, ib, k, out);
        }
    }
    int nc = (int)out.size();
    if (nc > cap) return -nc;
    if (nc) std::memcpy(outc, out.data(), sizeof(lpe_contact) * nc);
    return nc;
}

/* ---- PGS (contact_solver.cpp) ------------------------------------------ */
namespace {
struct Row {
    int a, b;           /* dynamic body slots or -1 */
    float dirX, dirY, rxA, ryA, rxB, ryB, effMass, rhs, lo, hi, lambda;
};

/* isInfiniteMass (contact_solver.cpp:42-47) */
bool infinite_mass(const lpe_body &b) { return (b.flags & LPE_BODY_HAS_MASS) && b.mass > 1e29; }
/* canRotate (:49-55) */
bool can_rotate(const lpe_body &b) {
    if (!(b.flags & LPE_BODY_HAS_ANGVEL) || !(b.flags & LPE_BODY_HAS_INERTIA)) return false;
    return b.inertia > 1e-12 && b.inertia < 1e29;
}
/* cross2fNeon (:207-214): (a.x*b.y) - (a.y*b.x), two products then a subtraction */
float cross2f(float ax, float ay, float bx, float by) {
    float l0 = ax * by, l1 = ay * bx;
    return l0 - l1;
}
}  // namespace

extern "C" int lpeo_pgs(const lpe_rigid_config *cfg, int nb, lpe_body *bodies, int nc,
                        const lpe_contact *contacts, const int32_t *order) {
    if (nc <= 0) return 0;
    /* buildBodyDOFTable (:70-98): every body in a contact; dynamic unless mass > 1e29 */
    std::vector<int> slot(nb, -2);
    std::vector<int> dyn;
    for (int k = 0; k < nc; k++) {
        for (int e : {contacts[k].a, contacts[k].b}) {
            if (slot[e] != -2) continue;
            if (!infinite_mass(bodies[e])) { slot[e] = (int)dyn.size(); dyn.push_back(e); }
            else slot[e] = -1;
        }
    }
    int nd = (int)dyn.size();
    std::vector<float> v(3 * (size_t)nd), im(nd), ii(nd);
    /* load (:480-507) */
    for (int i = 0; i < nd; i++) {
        const lpe_body &b = bodies[dyn[i]];
        double m = b.mass;
        im[i] = (m > 1e29) ? 0.f : (float)(1.0 / m);
        float iv = 0.f;
        if (can_rotate(b)) {
            double I = b.inertia;
            if (I > 1e-12 && I < 1e29) iv = (float)(1.0 / I);
        }
        ii[i] = iv;
        v[3 * i] = (float)b.vx;
        v[3 * i + 1] = (float)b.vy;
        v[3 * i + 2] = can_rotate(b) ? (float)b.omega : 0.f;
    }
    /* buildConstraintRows (:133-197) in solver order */
    std::vector<Row> rn(nc), rf(nc);
    for (int t = 0; t < nc; t++) {
        const lpe_contact &c = contacts[order ? order[t] : t];
        Row &n = rn[t];
        n.a = slot[c.a]; n.b = slot[c.b];
        V2 u = V2(c.nx, c.ny).normalized();
        n.dirX = (float)u.x; n.dirY = (float)u.y;
        const lpe_body &A = bodies[c.a], &B = bodies[c.b];
        n.rxA = (float)(c.px - A.x); n.ryA = (float)(c.py - A.y);
        n.rxB = (float)(c.px - B.x); n.ryB = (float)(c.py - B.y);
        n.lo = 0.0f; n.hi = 1e20f; n.lambda = 0.f; n.rhs = 0.0f; n.effMass = 0.0f;
        Row &f = rf[t];
        f = n;
        f.dirX = -n.dirY; f.dirY = n.dirX;
        f.lo = -1e20f; f.hi = 1e20f;
    }
    auto eff = [&](const Row &r) -> float {       /* computeEffectiveMass (:216-253) */
        float imA = 0.f, imB = 0.f, iiA = 0.f, iiB = 0.f;
        if (r.a >= 0) { imA = im[r.a]; iiA = ii[r.a]; }
        if (r.b >= 0) { imB = im[r.b]; iiB = ii[r.b]; }
        float rAxn = cross2f(r.rxA, r.ryA, r.dirX, r.dirY);
        float rBxn = cross2f(r.rxB, r.ryB, r.dirX, r.dirY);
        float sum = imA + imB + (rAxn * rAxn) * iiA + (rBxn * rBxn) * iiB;
        if (sum < 1e-12F) return 0.F;
        return 1.F / sum;
    };
    auto relv = [&](const Row &r) -> float {      /* getRelativeVelocity (:264-301) */
        float vxA = 0.f, vyA = 0.f, wA = 0.f, vxB = 0.f, vyB = 0.f, wB = 0.f;
        if (r.a >= 0) { vxA = v[3 * r.a]; vyA = v[3 * r.a + 1]; wA = v[3 * r.a + 2]; }
        if (r.b >= 0) { vxB = v[3 * r.b]; vyB = v[3 * r.b + 1]; wB = v[3 * r.b + 2]; }
        float ax = vxA - wA * r.ryA, ay = vyA + wA * r.rxA;
        float bx = vxB - wB * r.ryB, by = vyB + wB * r.rxB;
        float relX = bx - ax, relY = by - ay;
        return relX * r.dirX + relY * r.dirY;
    };
    auto apply = [&](const Row &r, float dl) {    /* applyImpulse (:315-356) */
        if (std::fabs(dl) < 1e-15F) return;
        if (r.a >= 0) {
            float imA = im[r.a], iiA = ii[r.a];
            v[3 * r.a] -= r.dirX * (dl * imA);
            v[3 * r.a + 1] -= r.dirY * (dl * imA);
            float crossA = r.rxA * r.dirY - r.ryA * r.dirX;
            v[3 * r.a + 2] -= crossA * dl * iiA;
        }
        if (r.b >= 0) {
            float imB = im[r.b], iiB = ii[r.b];
            v[3 * r.b] += r.dirX * (dl * imB);
            v[3 * r.b + 1] += r.dirY * (dl * imB);
            float crossB = r.rxB * r.dirY - r.ryB * r.dirX;
            v[3 * r.b + 2] += crossB * dl * iiB;
        }
    };
    /* solveLcpPgs (:381-440) */
    for (int t = 0; t < nc; t++) { rn[t].effMass = eff(rn[t]); rf[t].effMass = eff(rf[t]); }
    for (int it = 0; it < cfg->pgsIterations; ++it) {
        for (int t = 0; t < nc; t++) {
            {
                Row &r = rn[t];
                float vn = relv(r);
                float old = r.lambda;
                float dl = -r.effMass * (vn + r.rhs);
                float nl = old + dl;
                if (nl < r.lo) nl = r.lo;
                if (nl > r.hi) nl = r.hi;
                dl = nl - old;
                r.lambda = nl;
                apply(r, dl);
            }
            {
                Row &r = rf[t];
                float vt = relv(r);
                float old = r.lambda;
                float limit = cfg->frictionCoeff * rn[t].lambda;
                r.lo = -limit;
                r.hi = limit;
                float df = -r.effMass * (vt + r.rhs);
                float nf = old + df;
                if (nf < r.lo) nf = r.lo;
                if (nf > r.hi) nf = r.hi;
                df = nf - old;
                r.lambda = nf;
                apply(r, df);
            }
        }
    }
    /* write back (:516-529) */
    for (int i = 0; i < nd; i++) {
        lpe_body &b = bodies[dyn[i]];
        b.vx = v[3 * i];
        b.vy = v[3 * i + 1];
        if (can_rotate(b)) b.omega = v[3 * i + 2];
    }
    return nd;
}

/* ---- position solver (position_solver.cpp) ----------------------------- */
extern "C" int lpeo_position_solver(const lpe_rigid_config *cfg, int nb, lpe_body *bodies, int nc,
                                    const lpe_contact *contacts, const int32_t *order) {
    struct BD { bool valid, canRotate, isSolid; double invMass, invI, x, y, angle; };
    std::vector<int> slot(nb, -1);
    std::vector<int> ids;
    std::vector<int> corder;
    /* gatherPositionData (:67-120): skip contacts where neither body is Solid */
    for (int t = 0; t < nc; t++) {
        const lpe_contact &c = contacts[order ? order[t] : t];
        bool aS = (bodies[c.a].flags & LPE_BODY_HAS_PHASE) && is_solid(bodies[c.a]);
        bool bS = (bodies[c.b].flags & LPE_BODY_HAS_PHASE) && is_solid(bodies[c.b]);
        if (!aS && !bS) continue;
        for (int e : {c.a, c.b})
            if (slot[e] < 0) { slot[e] = (int)ids.size(); ids.push_back(e); }
        corder.push_back(order ? order[t] : t);
    }
    if (corder.empty()) return 0;
    /* loadBodyData (:125-168) */
    std::vector<BD> bd(ids.size());
    for (size_t k = 0; k < ids.size(); k++) {
        const lpe_body &b = bodies[ids[k]];
        BD &d = bd[k];
        d.valid = (b.flags & LPE_BODY_HAS_MASS) != 0;
        d.x = b.x; d.y = b.y;
        d.invMass = (b.mass > 1e29) ? 0.0 : (1.0 / b.mass);
        d.angle = (b.flags & LPE_BODY_HAS_ANGPOS) ? b.angle : 0.0;
        d.canRotate = false;
        d.invI = 0.0;
        if (b.flags & LPE_BODY_HAS_INERTIA) {
            double I = b.inertia;
            if (I < 1e29 && I > 1e-12) { d.canRotate = true; d.invI = 1.0 / I; }
        }
        d.isSolid = (b.flags & LPE_BODY_HAS_PHASE) && is_solid(b);
    }
    /* solvePositionContactsOnce x iterations (:215-290) */
    for (int it = 0; it < cfg->posIterations; it++) {
        for (int ci : corder) {
            const lpe_contact &c = contacts[ci];
            BD &a = bd[slot[c.a]];
            BD &b = bd[slot[c.b]];
            if (!a.valid || !b.valid) continue;
            if (!a.isSolid && !b.isSolid) continue;
            double pen = c.pen - cfg->slop;
            if (pen <= 0.0) continue;
            V2 n = V2(c.nx, c.ny).normalized();
            double corr = cfg->baumgarte * pen;
            double invMA = a.invMass, invMB = b.invMass, invIA = a.invI, invIB = b.invI;
            V2 rA(c.px - a.x, c.py - a.y);
            V2 rB(c.px - b.x, c.py - b.y);
            double rAn = rA.cross(n), rBn = rB.cross(n);
            double denom = invMA + invMB + (rAn * rAn) * invIA + (rBn * rBn) * invIB;
            if (denom < 1e-12) continue;
            double sc = corr / denom;
            double dx = n.x * sc, dy = n.y * sc;
            a.x -= dx * invMA;
            a.y -= dy * invMA;
            if (a.canRotate) a.angle -= rAn * sc * invIA;
            b.x += dx * invMB;
            b.y += dy * invMB;
            if (b.canRotate) b.angle += rBn * sc * invIB;
        }
    }
    /* storeBodyData (:176-197) */
    for (size_t k = 0; k < ids.size(); k++) {
        const BD &d = bd[k];
        if (!d.valid) continue;
        lpe_body &b = bodies[ids[k]];
        b.x = d.x; b.y = d.y;
        if (d.canRotate && (b.flags & LPE_BODY_HAS_ANGPOS)) b.angle = d.angle;
    }
    return (int)ids.size();
}

/* The canonical solver order of the device path (lpe_rigid.hip k_pair_colour):
 * the pairs that produced contacts are edge-coloured so that no two pairs of
 * one colour share a movable body (finite mass or rotatable), by rounds: every
 * uncoloured pair claims its movable bodies with the priority (hash(p), p),
 * the lowest wins a body, and a pair that won all its bodies takes a colour
 * free on both: with more pairs than one solver slot (1024), the first free
 * colour of the first K = ceil(pairs / 960) in the rotation r = hash(p ^
 * 0x9e3779b9) * K >> 32 (colours r, r + 1, .. mod K), else the lowest free
 * colour; balanced colours of <= 1024 pairs are one solver slot each.
 * Visiting order: colour-major, pairs ascending inside a colour, each pair's contacts in narrowphase order.  The reference's PGS order is an
 * unordered_map's (contact_manager.cpp:169-245); pairs of one colour touch
 * disjoint movable bodies, so any order inside a colour is bit-identical.
 * contacts must be grouped by pair (narrowphase order).  Returns the number
 * of colours, or -1 if more than 64 would be needed. */
uint32_t colour_hash(uint32_t x) {                /* lpe_rigid.hip colour_hash */
    x ^= x >> 16; x *= 0x7feb352du;
    x ^= x >> 15; x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
constexpr int COLOUR_SLOT = 1024;                    /* lpe_rigid.hip SOLVE_TPB */

extern "C" int lpeo_colour_order(int nb, const lpe_body *bodies, int nc, const lpe_contact *cs,
                                 int32_t *order, int32_t *pair_colour, int npairs) {
    auto dep = [&](int i) {
        const lpe_body &b = bodies[i];
        bool inf = (b.flags & LPE_BODY_HAS_MASS) && b.mass > 1e29;
        bool rot = (b.flags & LPE_BODY_HAS_INERTIA) && b.inertia > 1e-12 && b.inertia < 1e29;
        return !inf || rot;
    };
    /* pairs with contacts: index, bodies, contact range */
    std::vector<int> pid, pa, pb, ps, pn;
    for (int k = 0; k < nc; k++) {
        if (k == 0 || cs[k].pair != cs[k - 1].pair) {
            pid.push_back(cs[k].pair); pa.push_back(cs[k].a); pb.push_back(cs[k].b);
            ps.push_back(k); pn.push_back(0);
        }
        pn.back()++;
    }
    int m = (int)pid.size();
    std::vector<int> col(m, -2);
    std::vector<unsigned long long> used(nb, 0ull);
    const unsigned long long NONE = ~0ull;
    std::vector<unsigned long long> claim(nb, NONE);
    auto prio = [&](int p) {
        return ((unsigned long long)colour_hash((uint32_t)p) << 32) | (uint32_t)p;
    };
    const int FILL = COLOUR_SLOT - COLOUR_SLOT / 16;
    const int K = m > COLOUR_SLOT ? std::min((m + FILL - 1) / FILL, 64) : 0;
    for (int left = m; left > 0;) {
        for (int q = 0; q < m; q++) {
            if (col[q] != -2) continue;
            if (dep(pa[q])) claim[pa[q]] = std::min(claim[pa[q]], prio(pid[q]));
            if (dep(pb[q])) claim[pb[q]] = std::min(claim[pb[q]], prio(pid[q]));
        }
        std::vector<int> won;
        for (int q = 0; q < m; q++) {
            if (col[q] != -2) continue;
            int a = dep(pa[q]) ? pa[q] : -1, b = dep(pb[q]) ? pb[q] : -1;
            if ((a < 0 || claim[a] == prio(pid[q])) && (b < 0 || claim[b] == prio(pid[q]))) {
                unsigned long long forb = (a >= 0 ? used[a] : 0ull) | (b >= 0 ? used[b] : 0ull);
                if (forb == ~0ull) return -1;
                int c = -1;
                if (K > 0) {                          /* the first free of the first K, rotated by r */
                    const uint32_t r = (uint32_t)(((unsigned long long)colour_hash((uint32_t)pid[q] ^ 0x9e3779b9u) *
                                                   (unsigned)K) >> 32);
                    for (int i = 0; i < K && c < 0; i++) {
                        const int k = (int)((r + (uint32_t)i) % (uint32_t)K);
                        if (!((forb >> k) & 1ull)) c = k;
                    }
                }
                if (c < 0) {
                    c = 0;
                    while (forb & (1ull << c)) c++;
                }
                col[q] = -3 - c;
                won.push_back(q);
            }
        }
        for (int q = 0; q < m; q++) {
            if (col[q] == -2 || col[q] <= -3) {
                if (dep(pa[q])) claim[pa[q]] = NONE;
                if (dep(pb[q])) claim[pb[q]] = NONE;
            }
        }
        for (int q : won) {
            int c = -3 - col[q];
            col[q] = c;
            if (dep(pa[q])) used[pa[q]] |= 1ull << c;
            if (dep(pb[q])) used[pb[q]] |= 1ull << c;
            left--;
        }
    }
    int ncol = 0;
    for (int q = 0; q < m; q++) ncol = std::max(ncol, col[q] + 1);
    int t = 0;
    for (int c = 0; c < ncol; c++)
        for (int q = 0; q < m; q++)
            if (col[q] == c)
                for (int j = 0; j < pn[q]; j++) order[t++] = ps[q] + j;
    if (pair_colour) {
        for (int p = 0; p < npairs; p++) pair_colour[p] = -1;
        for (int q = 0; q < m; q++) if (pid[q] >= 0 && pid[q] < npairs) pair_colour[pid[q]] = col[q];
    }
    return ncol;
}

/* The canonical solver order of the device path since round 3 (lpe_rigid.hip
 * k_stripe_setup / k_group_colour / k_pgs_stripes / k_pos_stripes): striped
 * Gauss-Seidel.
 *  - movable body: finite mass or rotatable (colour_dep); the movable bodies
 *    of the pairs with contacts take part;
 *  - stripes: x0, x1 = min, max of their x; span = max |x_a - x_b| over the
 *    pairs whose two bodies are movable; q = (x1 - x0) / span; S = 1 unless
 *    there are more than 1024 pairs with contacts and q >= 2, else
 *    min(64, floor(q)) rounded down to even; w = (x1 - x0) / S;
 *    stripe(b) = clamp(floor((x_b - x0) / w), 0, S - 1).  A pair whose two
 *    movable bodies lie more than one stripe apart (a rounding edge) makes it
 *    one stripe (S = 1);
 *  - groups: band j = stripes 2j and 2j + 1, seam j = the stripe pair
 *    2j + 1 | 2j + 2.  A pair whose movable bodies (none: stripe 0) lie in
 *    one band is in the band's group 2j, one across bands j | j + 1 in the
 *    seam's group 2j + 1;
 *  - each group coloured greedily: its pairs ascending, each takes the
 *    lowest colour free on its movable bodies (64 at most);
 *  - order: phase A (the bands, groups 0, 2, 4, ..) then phase B (the seams,
 *    groups 1, 3, ..); per group its colours ascending, pairs ascending
 *    inside a colour, contacts in narrowphase order.
 * The bands touch disjoint bodies, and so do the seams: the device runs each
 * phase's groups concurrently (workgroup j: band j, then seam j, handing the
 * shared stripes 2j and 2j + 2 over with its neighbours), bit-identical to
 * this sequential order.  pair_step (optional, npairs)
 * receives the canonical step (group colour) of each pair, -1 without
 * contacts.  Returns the number of steps, or -1 (a group needs > 64 colours). */
constexpr int STRIPES_MAX = 64;                       /* lpe_rigid.hip STRIPES_MAX */
constexpr int STRIPE_MIN_PAIRS = 1024;                /* lpe_rigid.hip STRIPE_MIN_PAIRS */
extern "C" int lpeo_stripe_order(int nb, const lpe_body *bodies, int nc, const lpe_contact *cs,
                                 int32_t *order, int32_t *pair_step, int npairs, int32_t *nstripes) {
    auto dep = [&](int i) {
        const lpe_body &b = bodies[i];
        bool inf = (b.flags & LPE_BODY_HAS_MASS) && b.mass > 1e29;
        bool rot = (b.flags & LPE_BODY_HAS_INERTIA) && b.inertia > 1e-12 && b.inertia < 1e29;
        return !inf || rot;
    };
    std::vector<int> pid, pa, pb, ps, pn;             /* pairs with contacts, ascending */
    for (int k = 0; k < nc; k++) {
        if (k == 0 || cs[k].pair != cs[k - 1].pair) {
            pid.push_back(cs[k].pair); pa.push_back(cs[k].a); pb.push_back(cs[k].b);
            ps.push_back(k); pn.push_back(0);
        }
        pn.back()++;
    }
    const int m = (int)pid.size();
    double x0 = 0.0, x1 = 0.0, span = 0.0;
    bool any = false;
    for (int q = 0; q < m; q++) {
        for (int e : {pa[q], pb[q]}) {
            if (!dep(e)) continue;
            const double x = bodies[e].x;
            if (!any) { x0 = x1 = x; any = true; }
            x0 = std::min(x0, x); x1 = std::max(x1, x);
        }
        if (dep(pa[q]) && dep(pb[q])) span = std::max(span, std::fabs(bodies[pa[q]].x - bodies[pb[q]].x));
    }
    int S = 1;
    const double qn = (x1 - x0) / span;               /* (span 0: +inf; x1 == x0: 0 or NaN) */
    if (any && x1 > x0 && m > STRIPE_MIN_PAIRS && qn >= 2.0)
        S = std::min(STRIPES_MAX, (int)std::floor(std::min(qn, 1e9))) & ~1;
    const double w = (x1 - x0) / S;
    auto stripe = [&](int e) {
        if (S == 1) return 0;
        double f = std::floor((bodies[e].x - x0) / w);
        return (int)std::min((double)(S - 1), std::max(0.0, f));
    };
    for (int q = 0; q < m && S > 1; q++)
        if (dep(pa[q]) && dep(pb[q]) && std::abs(stripe(pa[q]) - stripe(pb[q])) > 1) S = 1;
    std::vector<int> grp(m);
    for (int q = 0; q < m; q++) {
        const bool da = dep(pa[q]), db = dep(pb[q]);
        int sa = da ? stripe(pa[q]) : -1, sb = db ? stripe(pb[q]) : -1;
        if (sa < 0) sa = sb;
        if (sb < 0) sb = sa;
        if (sa < 0) sa = sb = 0;
        grp[q] = (sa >> 1) == (sb >> 1) ? 2 * (sa >> 1) : 2 * (std::min(sa, sb) >> 1) + 1;
    }
    /* greedy colouring per group, pairs ascending */
    const int G = S;                                  /* bands 0, 2, .., seams 1, 3, .. */
    std::vector<int> col(m, -1), ncol(G, 0);
    std::vector<unsigned long long> used(nb, 0ull);
    for (int g = 0; g < G; g++) {
        std::vector<int> touched;
        for (int q = 0; q < m; q++) {
            if (grp[q] != g) continue;
            const int a = dep(pa[q]) ? pa[q] : -1, b = dep(pb[q]) ? pb[q] : -1;
            const unsigned long long forb = (a >= 0 ? used[a] : 0ull) | (b >= 0 ? used[b] : 0ull);
            if (forb == ~0ull) return -1;
            int c = 0;
            while (forb & (1ull << c)) c++;
            col[q] = c;
            ncol[g] = std::max(ncol[g], c + 1);
            if (a >= 0) { used[a] |= 1ull << c; touched.push_back(a); }
            if (b >= 0) { used[b] |= 1ull << c; touched.push_back(b); }
        }
        for (int e : touched) used[e] = 0ull;
    }
    /* canonical step sequence */
    std::vector<int> stepOf(G * 64, -1);
    int steps = 0;
    for (int ph = 0; ph < 2; ph++)
        for (int g = ph; g < G; g += 2)
            for (int c = 0; c < ncol[g]; c++) stepOf[g * 64 + c] = steps++;
    std::vector<std::vector<int>> bystep(steps);
    for (int q = 0; q < m; q++) bystep[stepOf[grp[q] * 64 + col[q]]].push_back(q);
    int t = 0;
    for (int k = 0; k < steps; k++)
        for (int q : bystep[k])
            for (int j = 0; j < pn[q]; j++) order[t++] = ps[q] + j;
    if (pair_step) {
        for (int p = 0; p < npairs; p++) pair_step[p] = -1;
        for (int q = 0; q < m; q++)
            if (pid[q] >= 0 && pid[q] < npairs) pair_step[pid[q]] = stepOf[grp[q] * 64 + col[q]];
    }
    if (nstripes) *nstripes = S;
    return steps;
}

extern "C" int lpeo_rigid_update(const lpe_rigid_config *cfg, int nb, lpe_body *bodies,
                                 const double *verts, lpeo_rigid_stats *st) {
    std::vector<int32_t> pairs(2 * 1024);
    int np = lpeo_broadphase(cfg, nb, bodies, verts, pairs.data(), 1024);
    if (np < 0) {
        pairs.resize(2 * (size_t)(-np));
        np = lpeo_broadphase(cfg, nb, bodies, verts, pairs.data(), -np);
    }
    std::vector<lpe_contact> cs(std::max(4 * np, 16));
    int nc = lpeo_narrowphase(nb, bodies, verts, np, pairs.data(), cs.data(), (int)cs.size());
    if (nc < 0) {
        cs.resize(-nc);
        nc = lpeo_narrowphase(nb, bodies, verts, np, pairs.data(), cs.data(), -nc);
    }
    if (st) { st->pairs = np; st->contacts = nc; st->manifolds = 0; st->dynamicBodies = 0; }
    if (nc == 0) return 0;   /* rigid_body_collision.cpp:35-37 */
    std::vector<int32_t> order(nc);
    if (lpeo_stripe_order(nb, bodies, nc, cs.data(), order.data(), nullptr, 0, nullptr) < 0)
        return -1;
    int nd = lpeo_pgs(cfg, nb, bodies, nc, cs.data(), order.data());
    lpeo_position_solver(cfg, nb, bodies, nc, cs.data(), order.data());
    if (st) {
        st->dynamicBodies = nd;
        int m = 0;
        for (int k = 0; k < nc; k++) if (k == 0 || cs[k].pair != cs[k - 1].pair) m++;
        st->manifolds = m;
    }
    return nc;
}

/* ---- integrators ------------------------------------------------------- */
extern "C" void lpeo_boundary(const lpe_rigid_config *cfg, int nb, lpe_body *bodies) {
    /* BoundarySystem::update (boundary.cpp:13-70) */
    const double m = cfg->marginPixels * cfg->metersPerPixel;
    const double U = cfg->universeSize;
    for (int i = 0; i < nb; i++) {
        lpe_body &b = bodies[i];
        if (!(b.flags & LPE_BODY_HAS_VEL)) continue;
        if ((b.flags & LPE_BODY_HAS_SLEEP) && (b.flags & LPE_BODY_ASLEEP)) continue;
        bool bounced = false;
        if (b.x < m) { b.x = m; b.vx = std::abs(b.vx) * cfg->bounceDamping; bounced = true; }
        else if (b.x > U - m) { b.x = U - m; b.vx = -std::abs(b.vx) * cfg->bounceDamping; bounced = true; }
        if (b.y < m) { b.y = m; b.vy = std::abs(b.vy) * cfg->bounceDamping; bounced = true; }
        else if (b.y > U - m) { b.y = U - m; b.vy = -std::abs(b.vy) * cfg->bounceDamping; bounced = true; }
        if (bounced) {
            double sp = std::sqrt(b.vx * b.vx + b.vy * b.vy);
            if (sp > cfg->maxSpeed) { b.vx = (b.vx / sp) * cfg->maxSpeed; b.vy = (b.vy / sp) * cfg->maxSpeed; }
        }
    }
}

extern "C" void lpeo_gravity(const lpe_rigid_config *cfg, int nb, lpe_body *bodies, double dt) {
    /* BasicGravitySystem::update (gravity.cpp:19-58) */
    auto inview = [](const lpe_body &b) {
        return (b.flags & LPE_BODY_HAS_PHASE) && (b.flags & LPE_BODY_HAS_VEL) &&
               (b.flags & LPE_BODY_HAS_MASS) && !(b.flags & LPE_BODY_BOUNDARY);
    };
    if (cfg->planetaryMassThreshold > 0.0)
        for (int i = 0; i < nb; i++)
            if (inview(bodies[i]) && bodies[i].mass >= cfg->planetaryMassThreshold) return;
    for (int i = 0; i < nb; i++)
        if (inview(bodies[i])) bodies[i].vy += cfg->gravity * dt;
}

extern "C" void lpeo_rotation(const lpe_rigid_config *cfg, int nb, lpe_body *bodies, double dt) {
    /* RotationSystem::update (rotation.cpp:18-60); Pi = 3.141592654 (constants.cpp:7) */
    const double Pi = 3.141592654;
    for (int i = 0; i < nb; i++) {
        lpe_body &b = bodies[i];
        if (!(b.flags & LPE_BODY_HAS_ANGPOS) || !(b.flags & LPE_BODY_HAS_ANGVEL)) continue;
        if (b.flags & LPE_BODY_BOUNDARY) continue;
        b.angle += b.omega * dt;
        if (cfg->angularDamping < 1.0) b.omega *= cfg->angularDamping;
        if (cfg->maxAngularSpeed > 0) {
            if (b.omega > cfg->maxAngularSpeed) b.omega = cfg->maxAngularSpeed;
            if (b.omega < -cfg->maxAngularSpeed) b.omega = -cfg->maxAngularSpeed;
        }
        if (b.angle > 2.0 * Pi) b.angle -= 2.0 * Pi;
        else if (b.angle < 0) b.angle += 2.0 * Pi;
    }
}

extern "C" void lpeo_movement(int nb, lpe_body *bodies, double dt) {
    /* MovementSystem::update (movement.cpp:13-39): skips Boundary and Liquid */
    for (int i = 0; i < nb; i++) {
        lpe_body &b = bodies[i];
        if (!(b.flags & LPE_BODY_HAS_VEL) || (b.flags & LPE_BODY_BOUNDARY)) continue;
        if ((b.flags & LPE_BODY_HAS_PHASE) && (b.flags & LPE_BODY_LIQUID)) continue;
        b.x += b.vx * dt;
        b.y += b.vy * dt;
    }
}

extern "C" void lpeo_sleep(const lpe_rigid_config *cfg, int nb, lpe_body *bodies) {
    /* SleepSystem::update (sleep.cpp:19-67) */
    for (int i = 0; i < nb; i++) {
        lpe_body &b = bodies[i];
        const uint32_t need = LPE_BODY_HAS_VEL | LPE_BODY_HAS_PHASE | LPE_BODY_HAS_MASS | LPE_BODY_HAS_SLEEP;
        if ((b.flags & need) != need) continue;
        if (b.flags & LPE_BODY_BOUNDARY) continue;
        double speed = std::sqrt(b.vx * b.vx + b.vy * b.vy);
        double ang = (b.flags & LPE_BODY_HAS_ANGVEL) ? std::fabs(b.omega) : 0.0;
        bool asleep = (b.flags & LPE_BODY_ASLEEP) != 0;
        if (speed < cfg->linearSleepThreshold && ang < cfg->angularSleepThreshold) {
            if (!asleep) {
                b.sleep_counter++;
                if (b.sleep_counter > cfg->sleepFramesThreshold) asleep = true;
            }
        } else {
            b.sleep_counter = 0;
            asleep = false;
        }
        if (asleep) {
            b.flags |= LPE_BODY_ASLEEP;
            b.vx = 0; b.vy = 0;
            if (b.flags & LPE_BODY_HAS_ANGVEL) b.omega = 0;
        } else {
            b.flags &= ~LPE_BODY_ASLEEP;
        }
    }
}

extern "C" int lpeo_rigid_tick(const lpe_rigid_config *cfg, int nb, lpe_body *bodies,
                               const double *verts, double dt_state, double dt_move,
                               lpeo_rigid_stats *stats) {
    lpeo_boundary(cfg, nb, bodies);
    lpeo_gravity(cfg, nb, bodies, dt_state);
    int nc = lpeo_rigid_update(cfg, nb, bodies, verts, stats);
    lpeo_rotation(cfg, nb, bodies, dt_state);
    lpeo_movement(nb, bodies, dt_move);
    lpeo_sleep(cfg, nb, bodies);
    return nc;
}

/* ---- the whole tick (ECSSimulator::tick, src/sim.cpp:156-163) ----------- */
#include "sph_oracle.h"

/* gatherRigidBodies (fluid.cpp:304-438) from a body */
static lpe_gpu_rigid gather_rigid(const lpe_body &b, const double *verts) {
    lpe_gpu_rigid rb;
    std::memset(&rb, 0, sizeof(rb));
    rb.posX = (float)b.x;
    rb.posY = (float)b.y;
    rb.angle = (b.flags & LPE_BODY_HAS_ANGPOS) ? (float)b.angle : 0.0f;
    if (b.flags & LPE_BODY_HAS_VEL) { rb.vx = (float)b.vx; rb.vy = (float)b.vy; }
    if (b.flags & LPE_BODY_HAS_ANGVEL) rb.omega = (float)b.omega;
    rb.mass = (b.flags & LPE_BODY_HAS_MASS) ? (float)b.mass : 1.f;
    rb.inertia = (b.flags & LPE_BODY_HAS_INERTIA) ? (float)b.inertia : 1.f;
    rb.minX = rb.posX - 0.5f; rb.maxX = rb.posX + 0.5f;
    rb.minY = rb.posY - 0.5f; rb.maxY = rb.posY + 0.5f;
    if (b.flags & LPE_BODY_CIRCLE) {
        rb.shapeType = 0;
        rb.radius = (float)b.radius;
        rb.minX = rb.posX - rb.radius; rb.maxX = rb.posX + rb.radius;
        rb.minY = rb.posY - rb.radius; rb.maxY = rb.posY + rb.radius;
    } else {
        rb.shapeType = 1;
        int cnt = std::min(b.vert_cnt, (int)LPE_MAX_POLY_VERTS);
        rb.vertCount = cnt;
        /* std::cos(float) (fluid.cpp:399-400: rb.angle is a float) */
        double c = (double)ocosf(rb.angle), s = (double)osinf(rb.angle);
        float mnx = FLT_MAX, mxx = -FLT_MAX, mny = FLT_MAX, mxy = -FLT_MAX;
        const double *lv = verts + 2 * (size_t)b.vert_off;
        for (int i = 0; i < cnt; i++) {
            double wx = b.x + (lv[2 * i] * c - lv[2 * i + 1] * s);
            double wy = b.y + (lv[2 * i] * s + lv[2 * i + 1] * c);
            rb.vertsX[i] = (float)wx;
            rb.vertsY[i] = (float)wy;
            if (wx < mnx) mnx = (float)wx;
            if (wx > mxx) mxx = (float)wx;
            if (wy < mny) mny = (float)wy;
            if (wy > mxy) mxy = (float)wy;
        }
        rb.minX = mnx; rb.maxX = mxx; rb.minY = mny; rb.maxY = mxy;
    }
    return rb;
}

extern "C" int lpeo_world_tick(const lpe_fluid_config *fcfg, const lpe_rigid_config *rcfg,
                               double spt, double time_accel, double bta, double ts,
                               lpeo_particle *parts, int n, lpe_body *bodies, int nb,
                               const double *verts, int nr, const int32_t *couple) {
    const double dt_fluid = spt * time_accel, dt_move = spt * time_accel, dt_state = spt * bta * ts;
    /* 1) FluidSystem::update */
    if (n > 0) {
        std::vector<lpe_gpu_rigid> rig(std::max(nr, 1));
        for (int r = 0; r < nr; r++) rig[r] = gather_rigid(bodies[couple[r]], verts);
        lpeo_fluid_tick(fcfg, dt_fluid, parts, n, rig.data(), nr, nullptr, nullptr);
        for (int r = 0; r < nr; r++) {                       /* fluid.cpp:564-579 */
            lpe_body &b = bodies[couple[r]];
            if (b.flags & LPE_BODY_HAS_VEL) { b.vx = rig[r].vx; b.vy = rig[r].vy; }
            if (b.flags & LPE_BODY_HAS_ANGVEL) b.omega = rig[r].omega;
        }
    }
    /* 2) Boundary, 3) Gravity: bodies, and fluid through the double ECS */
    lpeo_boundary(rcfg, nb, bodies);
    bool heavy = false;
    for (int i = 0; i < nb; i++) {
        const lpe_body &b = bodies[i];
        if ((b.flags & LPE_BODY_HAS_PHASE) && (b.flags & LPE_BODY_HAS_VEL) && (b.flags & LPE_BODY_HAS_MASS) &&
            !(b.flags & LPE_BODY_BOUNDARY) && rcfg->planetaryMassThreshold > 0.0 &&
            b.mass >= rcfg->planetaryMassThreshold)
            heavy = true;
    }
    for (int i = 0; i < n && rcfg->planetaryMassThreshold > 0.0; i++)
        if (parts[i].mass >= rcfg->planetaryMassThreshold) heavy = true;
    const double m = rcfg->marginPixels * rcfg->metersPerPixel, U = rcfg->universeSize;
    for (int i = 0; i < n; i++) {
        lpeo_particle &p = parts[i];
        double x = p.x, y = p.y, vx = p.vx, vy = p.vy;
        bool bounced = false;
        if (x < m) { x = m; vx = std::abs(vx) * rcfg->bounceDamping; bounced = true; }
        else if (x > U - m) { x = U - m; vx = -std::abs(vx) * rcfg->bounceDamping; bounced = true; }
        if (y < m) { y = m; vy = std::abs(vy) * rcfg->bounceDamping; bounced = true; }
        else if (y > U - m) { y = U - m; vy = -std::abs(vy) * rcfg->bounceDamping; bounced = true; }
        if (bounced) {
            double sp = std::sqrt(vx * vx + vy * vy);
            if (sp > rcfg->maxSpeed) { vx = (vx / sp) * rcfg->maxSpeed; vy = (vy / sp) * rcfg->maxSpeed; }
        }
        if (!heavy) vy += rcfg->gravity * dt_state;
        p.x = (float)x; p.y = (float)y; p.vx = (float)vx; p.vy = (float)vy;
    }
    if (!heavy)
        for (int i = 0; i < nb; i++) {
            lpe_body &b = bodies[i];
            if ((b.flags & LPE_BODY_HAS_PHASE) && (b.flags & LPE_BODY_HAS_VEL) &&
                (b.flags & LPE_BODY_HAS_MASS) && !(b.flags & LPE_BODY_BOUNDARY))
                b.vy += rcfg->gravity * dt_state;
        }
    /* 4) RigidBodyCollisionSystem, 6) Rotation, 7) Movement, 8) Sleep */
    lpeo_rigid_update(rcfg, nb, bodies, verts, nullptr);
    lpeo_rotation(rcfg, nb, bodies, dt_state);
    lpeo_movement(nb, bodies, dt_move);
    lpeo_sleep(rcfg, nb, bodies);
    return 0;
}

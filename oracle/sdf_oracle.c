/*
 * oracle/sdf_oracle.c -- TEST INFRASTRUCTURE: CPU restatement of how the reference fills its
 * distance field (StompCollisionSpace::setStartState, stomp_collision_space.cpp:154-197).
 * Paths are relative to /root/reference/stomp_motion_planner/.  Only tests/ load this.
 *
 *  1. Environment objects (addCollisionObjectsToPoints, :199-297).  A box or cylinder with an
 *     arbitrary pose is sampled on the lattice x = xlow, xlow + res, ... (a running double sum,
 *     the loop bound `x <= xlow + dim + resolution_` re-evaluated every step, :255-257 and
 *     :283-285); a cylinder keeps the lattice points with sqrt(xdist^2 + ydist^2) <= radius
 *     (:262-266); every kept point p = position - (x, y, z) is mapped through the KDL frame
 *     f = Frame(Rotation::Quaternion(x, y, z, w), position) (:243-248, 267-270, 287-289).
 *     The "points" namespace (collision-map points) is taken as given (:205-211).  Meshes
 *     (:212-223) are out of scope.
 *  2. Robot bodies (addAllBodiesButExcludeLinksToPoints / getVoxelsInBody, :564-650): the
 *     lattice center + g * res around the body's bounding sphere, g from
 *     (int)((c - r - c) * (1/res)) to (int)((c + r - c) * (1/res)) (worldToGrid / gridToWorld,
 *     stomp_collision_space.h:230-241), a point kept when the body contains it.  The reference
 *     counts the crossings of a +z ray (:636-643); for the convex primitives (sphere, box,
 *     cylinder) an odd count is containment, restated here as geometric_shapes'
 *     Body::containsPoint with the pose from btMatrix3x3::setRotation (third party, not
 *     vendored: points exactly on a surface are parity unpinned).  A mesh (a robot link's, or an
 *     environment object of type MESH, :216-223, which takes the same getVoxelsInBody path)
 *     becomes bodies::ConvexMesh: the convex hull of its vertices, whose ray-crossing parity is
 *     containment in the hull; restated as "inside every supporting plane" (so_hull_planes), the
 *     lattice centred on the bounding sphere around the vertices' bounding-box centre.
 *  3. distance_field::PropagationDistanceField::addPointsToField (third party): every point
 *     marks the cell round((p - origin) * (1/res)) when all three indices are in [0, n); the
 *     field is the capped exact EDT to the marked cells, stored as min(d2, cap^2) with
 *     cap = ceil(max_expansion / res) and d2 the integer squared cell distance (the field's
 *     distance_square_; its distance is sqrt_table_[d2] = sqrt(d2) * res).  The reference's
 *     own propagation (a 26-neighbour closest-point wavefront) can differ from the exact EDT
 *     by a fraction of a cell far from the obstacles: PARITY UNPINNED.
 *
 * Every double operation rounds once (-ffp-contract=off, see Makefile), in the order the
 * reference's expressions are written.
 */
#include "stomp_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

enum { SHAPE_BOX = 0, SHAPE_CYLINDER = 1, BODY_SPHERE = 2, BODY_BOX = 3, BODY_CYLINDER = 4, BODY_MESH = 5 };

/* KDL Rotation::Quaternion(x, y, z, w) (orocos KDL frames.cpp), row-major */
static void kdl_rot_quaternion(double x, double y, double z, double w, double* R)
{
    const double x2 = x * x, y2 = y * y, z2 = z * z, w2 = w * w;
    R[0] = w2 + x2 - y2 - z2; R[1] = 2 * x * y - 2 * w * z; R[2] = 2 * x * z + 2 * w * y;
    R[3] = 2 * x * y + 2 * w * z; R[4] = w2 - x2 + y2 - z2; R[5] = 2 * y * z - 2 * w * x;
    R[6] = 2 * x * z - 2 * w * y; R[7] = 2 * y * z + 2 * w * x; R[8] = w2 - x2 - y2 + z2;
}

/* btMatrix3x3::setRotation(btQuaternion) (bullet LinearMath, BT_USE_DOUBLE_PRECISION) */
static void bt_rot_quaternion(double x, double y, double z, double w, double* M)
{
    const double d = x * x + y * y + z * z + w * w;
    const double s = 2.0 / d;
    const double xs = x * s, ys = y * s, zs = z * s;
    const double wx = w * xs, wy = w * ys, wz = w * zs;
    const double xx = x * xs, xy = x * ys, xz = x * zs;
    const double yy = y * ys, yz = y * zs, zz = z * zs;
    M[0] = 1.0 - (yy + zz); M[1] = xy - wz; M[2] = xz + wy;
    M[3] = xy + wz; M[4] = 1.0 - (xx + zz); M[5] = yz - wx;
    M[6] = xz - wy; M[7] = yz + wx; M[8] = 1.0 - (xx + yy);
}

typedef struct {
    int n[3];
    double o[3], inv_res;
    unsigned char* occ;
    long long marked;
} marker;

/* PropagationDistanceField::addPointsToField -> VoxelGrid::worldToGrid: round((loc - origin) *
 * oo_resolution) per axis, the point dropped unless every index is in [0, n) */
static void mark(marker* mk, double px, double py, double pz)
{
    const double p[3] = {px, py, pz};
    long long c[3];
    for (int a = 0; a < 3; ++a) {
        const double r = round((p[a] - mk->o[a]) * mk->inv_res);
        if (!(r >= 0.0 && r < (double)mk->n[a])) return;
        c[a] = (long long)r;
    }
    if (mk->occ) mk->occ[(c[0] * mk->n[1] + c[1]) * mk->n[2] + c[2]] = 1;
    ++mk->marked;
}

/* addCollisionObjectsToPoints, box (:272-293) and cylinder (:249-271) branches */
static void env_shape(marker* mk, const so_shape* s, double res)
{
    const double* pos = s->position;
    const double* d = s->dims;
    double R[9];
    kdl_rot_quaternion(s->orientation[0], s->orientation[1], s->orientation[2], s->orientation[3], R);
    const int cyl = s->type == SHAPE_CYLINDER;
    const double xlow = cyl ? pos[0] - d[0] : pos[0] - d[0] / 2.0;
    const double ylow = cyl ? pos[1] - d[0] : pos[1] - d[1] / 2.0;
    const double zlow = cyl ? pos[2] - d[1] / 2.0 : pos[2] - d[2] / 2.0;
    const double radius = d[0];
    for (double x = xlow; x <= (cyl ? xlow + d[0] * 2.0 + res : xlow + d[0] + res); x += res) {
        for (double y = ylow; y <= (cyl ? ylow + d[0] * 2.0 + res : ylow + d[1] + res); y += res) {
            for (double z = zlow; z <= (cyl ? zlow + d[1] + res : zlow + d[2] + res); z += res) {
                if (cyl) {
                    const double xdist = fabs(pos[0] - x);
                    const double ydist = fabs(pos[1] - y);
                    if (!(sqrt(xdist * xdist + ydist * ydist) <= radius)) continue;
                }
                const double p[3] = {pos[0] - x, pos[1] - y, pos[2] - z};
                double p2[3];
                for (int i = 0; i < 3; ++i)   /* KDL Frame * Vector */
                    p2[i] = R[3 * i + 0] * p[0] + R[3 * i + 1] * p[1] + R[3 * i + 2] * p[2] + pos[i];
                mark(mk, p2[0], p2[1], p2[2]);
            }
        }
    }
}

/* geometric_shapes bodies::{Sphere,Box,Cylinder}::containsPoint; v = p - center, n_k = basis
 * column k, v.dot(n) = v0 n0 + v1 n1 + v2 n2 (btVector3::dot) */
static double dotcol(const double* v, const double* B, int k)
{
    return v[0] * B[k] + v[1] * B[3 + k] + v[2] * B[6 + k];
}

/* Supporting planes of the convex hull of V (bodies::ConvexMesh's qhull hull, restated).
 *   1. Vertices with identical coordinates are merged (the first index kept): COLLADA meshes
 *      repeat positions.
 *   2. Incremental hull of the unique vertices in index order: a first tetrahedron (vertex 0, the
 *      one farthest from it, the one farthest from their line, the one farthest from their
 *      plane), then each vertex that lies more than eps outside some face replaces the faces it
 *      sees by a fan over their horizon (directed edges found through a hash of (a, b) -> face).
 *   3. Faces whose planes agree (n . n' > 1 - 1e-12, |d - d'| <= eps) form one facet; a facet's
 *      plane is spanned by the first triple i < j < k of its vertices (index order) that is not
 *      collinear (|u x w| > 1e-12 |u| |w|) and leaves every hull vertex within eps on one side,
 *      n = (vj - vi) x (vk - vi) / |.|, d = -(n . vi), flipped so the hull lies on the negative
 *      side.  Facets are emitted in the order of their triples, a plane equal to one already
 *      emitted (same normal and offset test) skipped.
 * eps = 1e-9 (1 + max |coordinate|).  O(V log V + V F) instead of the O(V^4) triple scan.  The
 * engine (csrc/engine.cpp hull_planes) implements the same steps in C++. */
typedef struct {
    int v[3];
    double n[3], d;
    int alive;
} hull_face;

typedef struct {
    unsigned long long* key;
    int* val;
    size_t cap, used;
} edge_map;

static size_t em_slot(const edge_map* m, unsigned long long k)
{
    size_t h = (size_t)((k * 0x9E3779B97F4A7C15ull) >> 17) & (m->cap - 1);
    while (m->val[h] >= 0 && m->key[h] != k) h = (h + 1) & (m->cap - 1);
    return h;
}

static int em_grow(edge_map* m)
{
    edge_map n = {0};
    n.cap = m->cap ? 2 * m->cap : 1024;
    n.key = (unsigned long long*)malloc(sizeof(unsigned long long) * n.cap);
    n.val = (int*)malloc(sizeof(int) * n.cap);
    if (!n.key || !n.val) { free(n.key); free(n.val); return -1; }
    for (size_t i = 0; i < n.cap; ++i) n.val[i] = -1;
    for (size_t i = 0; i < m->cap; ++i)
        if (m->val[i] >= 0) {
            const size_t h = em_slot(&n, m->key[i]);
            n.key[h] = m->key[i];
            n.val[h] = m->val[i];
            ++n.used;
        }
    free(m->key); free(m->val);
    *m = n;
    return 0;
}

static int em_put(edge_map* m, int a, int b, int f)
{
    if (2 * (m->used + 1) > m->cap && em_grow(m)) return -1;
    const unsigned long long k = ((unsigned long long)(unsigned)a << 32) | (unsigned)b;
    const size_t h = em_slot(m, k);
    if (m->val[h] < 0) ++m->used;
    m->key[h] = k;
    m->val[h] = f;
    return 0;
}

static int em_get(const edge_map* m, int a, int b)
{
    const unsigned long long k = ((unsigned long long)(unsigned)a << 32) | (unsigned)b;
    return m->val[em_slot(m, k)];
}

static const double* hv(const double* V, int i) { return V + 3 * (size_t)i; }

/* plane through vertices a, b, c: unit normal of (b - a) x (c - a) and offset; 0 when collinear */
static int plane3(const double* V, int a, int b, int c, double* n, double* d)
{
    const double* A = hv(V, a); const double* B = hv(V, b); const double* C = hv(V, c);
    const double u[3] = {B[0] - A[0], B[1] - A[1], B[2] - A[2]};
    const double w[3] = {C[0] - A[0], C[1] - A[1], C[2] - A[2]};
    n[0] = u[1] * w[2] - u[2] * w[1]; n[1] = u[2] * w[0] - u[0] * w[2]; n[2] = u[0] * w[1] - u[1] * w[0];
    const double len = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    const double lu = sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]), lw = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    if (!(len > 1e-12 * lu * lw) || !(len > 0.0)) return 0;
    n[0] /= len; n[1] /= len; n[2] /= len;
    *d = -(n[0] * A[0] + n[1] * A[1] + n[2] * A[2]);
    return 1;
}

static double sdist(const double* n, double d, const double* p) { return n[0] * p[0] + n[1] * p[1] + n[2] * p[2] + d; }

static const double* g_sort_v;
static int cmp_xyz(const void* a, const void* b)
{
    const int i = *(const int*)a, j = *(const int*)b;
    for (int k = 0; k < 3; ++k) {
        const double x = g_sort_v[3 * (size_t)i + k], y = g_sort_v[3 * (size_t)j + k];
        if (x < y) return -1;
        if (x > y) return 1;
    }
    return i < j ? -1 : (i > j);
}

static int cmp_int(const void* a, const void* b)
{
    const int i = *(const int*)a, j = *(const int*)b;
    return i < j ? -1 : (i > j);
}

typedef struct { int t[3]; double n[3], d; } hull_facet;

static int cmp_facet(const void* a, const void* b)
{
    const hull_facet* x = (const hull_facet*)a; const hull_facet* y = (const hull_facet*)b;
    for (int k = 0; k < 3; ++k)
        if (x->t[k] != y->t[k]) return x->t[k] < y->t[k] ? -1 : 1;
    return 0;
}

int so_hull_planes(const double* V, int nv, double* planes, int max_planes)
{
    if (nv < 4) return -1;
    double ext = 0.0;
    for (int i = 0; i < 3 * nv; ++i)
        if (fabs(V[i]) > ext) ext = fabs(V[i]);
    const double eps = 1e-9 * (1.0 + ext);
    int rc = -1, nu = 0, nf = 0, capf = 0, nh = 0;
    int* ord = (int*)malloc(sizeof(int) * (size_t)nv);
    int* uq = (int*)malloc(sizeof(int) * (size_t)nv);
    unsigned char* onhull = (unsigned char*)calloc((size_t)nv, 1);
    int* hullv = (int*)malloc(sizeof(int) * (size_t)nv);
    hull_face* F = NULL;
    hull_facet* fc = NULL;
    int *vis = NULL, *hor = NULL, *grp = NULL, *fv = NULL;
    edge_map em = {0};
    if (!ord || !uq || !onhull || !hullv) goto done;
    /* 1. unique vertices */
    for (int i = 0; i < nv; ++i) ord[i] = i;
    g_sort_v = V;
    qsort(ord, (size_t)nv, sizeof(int), cmp_xyz);
    for (int i = 0; i < nv; ++i) {
        const double* p = hv(V, ord[i]);
        if (i > 0) {
            const double* q = hv(V, ord[i - 1]);
            if (p[0] == q[0] && p[1] == q[1] && p[2] == q[2]) continue;   /* the group's first index came first */
        }
        uq[nu++] = ord[i];
    }
    qsort(uq, (size_t)nu, sizeof(int), cmp_int);
    if (nu < 4) goto done;
    /* 2. the first tetrahedron */
    {
        const int a = uq[0];
        int b = -1, c = -1, e = -1;
        double best = eps;
        for (int i = 1; i < nu; ++i) {
            const double* p = hv(V, uq[i]); const double* A = hv(V, a);
            const double dx = p[0] - A[0], dy = p[1] - A[1], dz = p[2] - A[2];
            const double r = sqrt(dx * dx + dy * dy + dz * dz);
            if (r > best) { best = r; b = uq[i]; }
        }
        if (b < 0) goto done;
        best = eps;
        for (int i = 1; i < nu; ++i) {
            const double* A = hv(V, a); const double* B = hv(V, b); const double* p = hv(V, uq[i]);
            const double u[3] = {B[0] - A[0], B[1] - A[1], B[2] - A[2]};
            const double w[3] = {p[0] - A[0], p[1] - A[1], p[2] - A[2]};
            const double x[3] = {u[1] * w[2] - u[2] * w[1], u[2] * w[0] - u[0] * w[2], u[0] * w[1] - u[1] * w[0]};
            const double r = sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]) / sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
            if (r > best) { best = r; c = uq[i]; }
        }
        if (c < 0) goto done;
        double n[3], d;
        if (!plane3(V, a, b, c, n, &d)) goto done;
        best = eps;
        for (int i = 1; i < nu; ++i) {
            const double r = fabs(sdist(n, d, hv(V, uq[i])));
            if (r > best) { best = r; e = uq[i]; }
        }
        if (e < 0) goto done;
        const int tet[4][3] = {{a, b, c}, {a, e, b}, {b, e, c}, {c, e, a}};
        double ctr[3];
        for (int k = 0; k < 3; ++k) ctr[k] = (hv(V, a)[k] + hv(V, b)[k] + hv(V, c)[k] + hv(V, e)[k]) / 4.0;
        capf = 64;
        F = (hull_face*)malloc(sizeof(hull_face) * (size_t)capf);
        if (!F) goto done;
        for (int f = 0; f < 4; ++f) {
            hull_face* h = &F[nf++];
            h->v[0] = tet[f][0]; h->v[1] = tet[f][1]; h->v[2] = tet[f][2];
            if (!plane3(V, h->v[0], h->v[1], h->v[2], h->n, &h->d)) goto done;
            if (sdist(h->n, h->d, ctr) > 0.0) {   /* orient outward */
                const int t = h->v[1]; h->v[1] = h->v[2]; h->v[2] = t;
                if (!plane3(V, h->v[0], h->v[1], h->v[2], h->n, &h->d)) goto done;
            }
            h->alive = 1;
            for (int k = 0; k < 3; ++k)
                if (em_put(&em, h->v[k], h->v[(k + 1) % 3], f)) goto done;
        }
        onhull[a] = onhull[b] = onhull[c] = onhull[e] = 1;
    }
    /* the rest, in index order */
    vis = (int*)malloc(sizeof(int) * 16);
    hor = (int*)malloc(sizeof(int) * 32);
    int capv = 16, caph = 16;
    if (!vis || !hor) goto done;
    for (int i = 1; i < nu; ++i) {
        const int p = uq[i];
        if (onhull[p]) continue;
        const double* P = hv(V, p);
        int nvis = 0;
        for (int f = 0; f < nf; ++f) {
            if (!F[f].alive || !(sdist(F[f].n, F[f].d, P) > eps)) continue;
            if (nvis == capv) { capv *= 2; int* t = (int*)realloc(vis, sizeof(int) * (size_t)capv); if (!t) goto done; vis = t; }
            vis[nvis++] = f;
        }
        if (!nvis) continue;   /* inside, or within eps of the hull */
        for (int q = 0; q < nvis; ++q) F[vis[q]].alive = 2;   /* visible */
        int nhor = 0;
        for (int q = 0; q < nvis; ++q) {
            const hull_face* h = &F[vis[q]];
            for (int k = 0; k < 3; ++k) {
                const int ea = h->v[k], eb = h->v[(k + 1) % 3];
                const int o = em_get(&em, eb, ea);
                if (o >= 0 && F[o].alive == 2) continue;   /* interior edge of the visible region */
                if (nhor == caph) { caph *= 2; int* t = (int*)realloc(hor, sizeof(int) * 2 * (size_t)caph); if (!t) goto done; hor = t; }
                hor[2 * nhor] = ea; hor[2 * nhor + 1] = eb; ++nhor;
            }
        }
        for (int q = 0; q < nvis; ++q) F[vis[q]].alive = 0;
        for (int q = 0; q < nhor; ++q) {
            if (nf == capf) { capf *= 2; hull_face* t = (hull_face*)realloc(F, sizeof(hull_face) * (size_t)capf); if (!t) goto done; F = t; }
            hull_face* h = &F[nf];
            h->v[0] = hor[2 * q]; h->v[1] = hor[2 * q + 1]; h->v[2] = p;
            h->alive = 1;
            if (!plane3(V, h->v[0], h->v[1], h->v[2], h->n, &h->d)) { h->n[0] = h->n[1] = h->n[2] = 0.0; h->d = 0.0; }
            for (int k = 0; k < 3; ++k)
                if (em_put(&em, h->v[k], h->v[(k + 1) % 3], nf)) goto done;
            ++nf;
        }
        onhull[p] = 1;
    }
    /* 3. facets: faces grouped by plane, each facet's plane from its first spanning triple */
    for (int f = 0; f < nf; ++f)
        if (F[f].alive)
            for (int k = 0; k < 3; ++k) onhull[F[f].v[k]] = 2;
    for (int i = 0; i < nu; ++i)
        if (onhull[uq[i]] == 2) hullv[nh++] = uq[i];
    grp = (int*)malloc(sizeof(int) * (size_t)nf);
    fv = (int*)malloc(sizeof(int) * 3 * (size_t)nf);
    fc = (hull_facet*)malloc(sizeof(hull_facet) * (size_t)nf);
    if (!grp || !fv || !fc) goto done;
    for (int f = 0; f < nf; ++f) grp[f] = -1;
    int nfc = 0;
    for (int f = 0; f < nf; ++f) {
        if (!F[f].alive || grp[f] >= 0) continue;
        int m = 0;
        for (int g = f; g < nf; ++g) {
            if (!F[g].alive || grp[g] >= 0) continue;
            if (g != f && !(F[f].n[0] * F[g].n[0] + F[f].n[1] * F[g].n[1] + F[f].n[2] * F[g].n[2] > 1.0 - 1e-12 &&
                            fabs(F[f].d - F[g].d) <= eps))
                continue;
            grp[g] = f;
            for (int k = 0; k < 3; ++k) fv[m++] = F[g].v[k];
        }
        qsort(fv, (size_t)m, sizeof(int), cmp_int);
        int mu = 0;
        for (int q = 0; q < m; ++q)
            if (!mu || fv[mu - 1] != fv[q]) fv[mu++] = fv[q];
        int found = 0;
        for (int x = 0; x < mu && !found; ++x)
            for (int y = x + 1; y < mu && !found; ++y)
                for (int z = y + 1; z < mu && !found; ++z) {
                    double n[3], d;
                    if (!plane3(V, fv[x], fv[y], fv[z], n, &d)) continue;
                    double smax = -1e300, smin = 1e300;
                    for (int q = 0; q < nh; ++q) {
                        const double sd = sdist(n, d, hv(V, hullv[q]));
                        if (sd > smax) smax = sd;
                        if (sd < smin) smin = sd;
                    }
                    if (smax <= eps) {
                    } else if (smin >= -eps) {
                        n[0] = -n[0]; n[1] = -n[1]; n[2] = -n[2]; d = -d;
                    } else {
                        continue;
                    }
                    hull_facet* o = &fc[nfc++];
                    o->t[0] = fv[x]; o->t[1] = fv[y]; o->t[2] = fv[z];
                    o->n[0] = n[0]; o->n[1] = n[1]; o->n[2] = n[2]; o->d = d;
                    found = 1;
                }
    }
    qsort(fc, (size_t)nfc, sizeof(hull_facet), cmp_facet);
    int np = 0;
    for (int q = 0; q < nfc; ++q) {
        int dup = 0;
        for (int p2 = 0; p2 < np && !dup; ++p2) {
            const double* e = planes + 4 * p2;
            dup = fc[q].n[0] * e[0] + fc[q].n[1] * e[1] + fc[q].n[2] * e[2] > 1.0 - 1e-12 && fabs(fc[q].d - e[3]) <= eps;
        }
        if (dup) continue;
        if (np == max_planes) goto done;
        planes[4 * np] = fc[q].n[0]; planes[4 * np + 1] = fc[q].n[1]; planes[4 * np + 2] = fc[q].n[2];
        planes[4 * np + 3] = fc[q].d;
        ++np;
    }
    rc = np >= 4 ? np : -1;
done:
    free(ord); free(uq); free(onhull); free(hullv); free(F); free(fc); free(vis); free(hor); free(grp); free(fv);
    free(em.key); free(em.val);
    return rc;
}

/* the mesh body: centre of the vertices' bounding box and the largest distance of a vertex from
 * it (bodies::ConvexMesh's bounding sphere before the pose; third party, parity unpinned) */
static void mesh_box_sphere(const double* V, int nv, double* centre, double* radius)
{
    double lo[3] = {V[0], V[1], V[2]}, hi[3] = {V[0], V[1], V[2]};
    for (int q = 1; q < nv; ++q)
        for (int a = 0; a < 3; ++a) {
            if (V[3 * q + a] < lo[a]) lo[a] = V[3 * q + a];
            if (V[3 * q + a] > hi[a]) hi[a] = V[3 * q + a];
        }
    for (int a = 0; a < 3; ++a) centre[a] = (lo[a] + hi[a]) / 2.0;
    double r2 = 0.0;
    for (int q = 0; q < nv; ++q) {
        const double dx = V[3 * q] - centre[0], dy = V[3 * q + 1] - centre[1], dz = V[3 * q + 2] - centre[2];
        const double s = dx * dx + dy * dy + dz * dz;
        if (s > r2) r2 = s;
    }
    *radius = sqrt(r2);
}

static int body_contains(int type, const double* c, const double* B, const double* d, const double* p)
{
    const double v[3] = {p[0] - c[0], p[1] - c[1], p[2] - c[2]};
    if (type == BODY_SPHERE) {
        return v[0] * v[0] + v[1] * v[1] + v[2] * v[2] < d[0] * d[0];
    }
    if (type == BODY_BOX) {
        if (fabs(dotcol(v, B, 0)) > d[0] / 2.0) return 0;
        if (fabs(dotcol(v, B, 1)) > d[1] / 2.0) return 0;
        if (fabs(dotcol(v, B, 2)) > d[2] / 2.0) return 0;
        return 1;
    }
    /* cylinder: axis = basis z, radius d[0], length d[1] */
    if (fabs(dotcol(v, B, 2)) > d[1] / 2.0) return 0;
    const double b1 = dotcol(v, B, 0);
    const double remaining = d[0] * d[0] - b1 * b1;
    if (remaining < 0.0) return 0;
    const double b2 = dotcol(v, B, 1);
    return b2 * b2 < remaining;
}

/* bodies::*::computeBoundingSphere radius */
static double body_bounding_radius(int type, const double* d)
{
    if (type == BODY_SPHERE) return d[0];
    if (type == BODY_BOX) {
        const double a = d[0] / 2.0, b = d[1] / 2.0, c = d[2] / 2.0;
        return sqrt(a * a + b * b + c * c);
    }
    const double h = d[1] / 2.0;
    return sqrt(d[0] * d[0] + h * h);
}

/* getVoxelsInBody (:592-650) for a mesh: the lattice around the bounding sphere, a point kept
 * when, in the body frame (v = w - position, components v . basis column), it lies inside every
 * hull plane grown by the padding */
static int mesh_body(marker* mk, const so_shape* s, double res)
{
    if (!s->vertices || s->num_vertices < 4) return -1;
    const int nv = s->num_vertices;
    const int maxp = 2 * nv * nv + 8;
    double* planes = (double*)malloc(sizeof(double) * 4 * (size_t)maxp);
    const int np = so_hull_planes(s->vertices, nv, planes, maxp);
    if (np < 0) {
        free(planes);
        return -1;
    }
    double B[9];
    bt_rot_quaternion(s->orientation[0], s->orientation[1], s->orientation[2], s->orientation[3], B);
    double bc[3], rb;
    mesh_box_sphere(s->vertices, nv, bc, &rb);
    const double pad = s->dims[0];
    const double* pos = s->position;
    double c[3];
    for (int a = 0; a < 3; ++a) c[a] = B[3 * a] * bc[0] + B[3 * a + 1] * bc[1] + B[3 * a + 2] * bc[2] + pos[a];
    const double r = rb + pad;
    int lo[3], hi[3];
    for (int a = 0; a < 3; ++a) {
        lo[a] = (int)(((c[a] - r) - c[a]) * (1.0 / res));
        hi[a] = (int)(((c[a] + r) - c[a]) * (1.0 / res));
    }
    for (int x = lo[0]; x <= hi[0]; ++x)
        for (int y = lo[1]; y <= hi[1]; ++y)
            for (int z = lo[2]; z <= hi[2]; ++z) {
                const double w[3] = {x * res + c[0], y * res + c[1], z * res + c[2]};   /* gridToWorld */
                const double v[3] = {w[0] - pos[0], w[1] - pos[1], w[2] - pos[2]};
                const double pb[3] = {dotcol(v, B, 0), dotcol(v, B, 1), dotcol(v, B, 2)};
                int in = 1;
                for (int p = 0; p < np && in; ++p) {
                    const double* e = planes + 4 * p;
                    in = !(e[0] * pb[0] + e[1] * pb[1] + e[2] * pb[2] + e[3] > pad);
                }
                if (in) mark(mk, w[0], w[1], w[2]);
            }
    free(planes);
    return 0;
}

/* getVoxelsInBody (:592-650) */
static void robot_body(marker* mk, const so_shape* s, double res)
{
    const double* c = s->position;
    double B[9];
    bt_rot_quaternion(s->orientation[0], s->orientation[1], s->orientation[2], s->orientation[3], B);
    const double r = body_bounding_radius(s->type, s->dims);
    int lo[3], hi[3];
    for (int a = 0; a < 3; ++a) {   /* worldToGrid(center, c -/+ r): (int)((w - origin) * (1.0 / res)) */
        lo[a] = (int)(((c[a] - r) - c[a]) * (1.0 / res));
        hi[a] = (int)(((c[a] + r) - c[a]) * (1.0 / res));
    }
    for (int x = lo[0]; x <= hi[0]; ++x)
        for (int y = lo[1]; y <= hi[1]; ++y)
            for (int z = lo[2]; z <= hi[2]; ++z) {
                const double w[3] = {x * res + c[0], y * res + c[1], z * res + c[2]};   /* gridToWorld */
                if (body_contains(s->type, c, B, s->dims, w)) mark(mk, w[0], w[1], w[2]);
            }
}

/* exact EDT to the marked cells, capped: separable (1-D distances along z, then the minimum over
 * a window of |dy| <= cap along y and |dx| <= cap along x).  A window term needs its component
 * <= cap to reach a value <= cap^2, so the windowed minimum is exact wherever the result is
 * below the cap, and anything above is clamped to it. */
int so_sdf_from_occupancy(int nx, int ny, int nz, double res, double max_expansion, const unsigned char* occ,
                          unsigned short* sdf)
{
    const int cap = (int)ceil(max_expansion / res);
    if (cap < 0 || cap > 255) return -1;
    const long long cap2 = (long long)cap * cap, far = cap2 + 1;
    const size_t n = (size_t)nx * ny * nz;
    long long* a = (long long*)malloc(n * sizeof(long long));
    long long* b = (long long*)malloc(n * sizeof(long long));
    for (int x = 0; x < nx; ++x)
        for (int y = 0; y < ny; ++y) {
            const size_t base = ((size_t)x * ny + y) * nz;
            long long last = -1;
            for (int z = 0; z < nz; ++z) {   /* distance to the nearest marked cell at or below z */
                if (occ[base + z]) last = z;
                const long long dz = last < 0 ? cap + 1 : z - last;
                a[base + z] = dz > cap ? far : dz * dz;
            }
            last = -1;
            for (int z = nz - 1; z >= 0; --z) {   /* ... or above */
                if (occ[base + z]) last = z;
                const long long dz = last < 0 ? cap + 1 : last - z;
                const long long v = dz > cap ? far : dz * dz;
                if (v < a[base + z]) a[base + z] = v;
            }
        }
    for (int x = 0; x < nx; ++x)
        for (int y = 0; y < ny; ++y)
            for (int z = 0; z < nz; ++z) {
                long long best = far;
                for (int yy = y - cap < 0 ? 0 : y - cap; yy <= y + cap && yy < ny; ++yy) {
                    const long long v = a[((size_t)x * ny + yy) * nz + z] + (long long)(y - yy) * (y - yy);
                    if (v < best) best = v;
                }
                b[((size_t)x * ny + y) * nz + z] = best;
            }
    for (int x = 0; x < nx; ++x)
        for (int y = 0; y < ny; ++y)
            for (int z = 0; z < nz; ++z) {
                long long best = far;
                for (int xx = x - cap < 0 ? 0 : x - cap; xx <= x + cap && xx < nx; ++xx) {
                    const long long v = b[((size_t)xx * ny + y) * nz + z] + (long long)(x - xx) * (x - xx);
                    if (v < best) best = v;
                }
                const long long d2 = best < cap2 ? best : cap2;
                sdf[((size_t)x * ny + y) * nz + z] = (unsigned short)d2;
            }
    free(a);
    free(b);
    return 0;
}

long long so_sdf_build_objects(int nx, int ny, int nz, const double* origin, double res, double max_expansion,
                               const so_shape* shapes, int n_shapes, const double* points, long long n_points,
                               unsigned char* occ, unsigned short* sdf)
{
    if (nx <= 0 || ny <= 0 || nz <= 0 || !(res > 0)) return -1;
    if (sdf && !(ceil(max_expansion / res) <= 255.0)) return -1;
    const size_t n = (size_t)nx * ny * nz;
    unsigned char* own = NULL;
    if (!occ && sdf) occ = own = (unsigned char*)malloc(n);
    if (occ) memset(occ, 0, n);
    marker mk = {{nx, ny, nz}, {origin[0], origin[1], origin[2]}, 1.0 / res, occ, 0};
    for (long long i = 0; i < n_points; ++i) mark(&mk, points[3 * i], points[3 * i + 1], points[3 * i + 2]);
    for (int s = 0; s < n_shapes; ++s) {
        if (shapes[s].type == SHAPE_BOX || shapes[s].type == SHAPE_CYLINDER) env_shape(&mk, &shapes[s], res);
        else if (shapes[s].type >= BODY_SPHERE && shapes[s].type <= BODY_CYLINDER) robot_body(&mk, &shapes[s], res);
        else if (shapes[s].type == BODY_MESH) {
            if (mesh_body(&mk, &shapes[s], res) != 0) {
                free(own);
                return -1;
            }
        } else {
            free(own);
            return -1;
        }
    }
    if (sdf) so_sdf_from_occupancy(nx, ny, nz, res, max_expansion, occ, sdf);
    free(own);
    return mk.marked;
}

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

/* supporting planes of the convex hull of V: every vertex triple i < j < k in order spans a
 * candidate plane n = (vj - vi) x (vk - vi) / |.|, d = -(n . vi); it is kept (flipped so that
 * the hull lies on the negative side) when no vertex lies more than eps on each side of it,
 * unless a kept plane already has the same normal (n . n' > 1 - 1e-12) and offset (within eps).
 * eps = 1e-9 (1 + max |coordinate|).  Deterministic: the engine runs the same loops. */
int so_hull_planes(const double* V, int nv, double* planes, int max_planes)
{
    double ext = 0.0;
    for (int i = 0; i < 3 * nv; ++i)
        if (fabs(V[i]) > ext) ext = fabs(V[i]);
    const double eps = 1e-9 * (1.0 + ext);
    int np = 0;
    for (int i = 0; i < nv; ++i)
        for (int j = i + 1; j < nv; ++j)
            for (int k = j + 1; k < nv; ++k) {
                const double* a = V + 3 * i;
                const double* b = V + 3 * j;
                const double* c = V + 3 * k;
                const double u[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
                const double w[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
                double n[3] = {u[1] * w[2] - u[2] * w[1], u[2] * w[0] - u[0] * w[2], u[0] * w[1] - u[1] * w[0]};
                const double len = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
                if (!(len > eps * eps)) continue;   /* (nearly) collinear */
                n[0] /= len; n[1] /= len; n[2] /= len;
                double d = -(n[0] * a[0] + n[1] * a[1] + n[2] * a[2]);
                double smax = -1e300, smin = 1e300;
                for (int q = 0; q < nv; ++q) {
                    const double sd = n[0] * V[3 * q] + n[1] * V[3 * q + 1] + n[2] * V[3 * q + 2] + d;
                    if (sd > smax) smax = sd;
                    if (sd < smin) smin = sd;
                }
                if (smax <= eps) {
                    /* hull below the plane */
                } else if (smin >= -eps) {
                    n[0] = -n[0]; n[1] = -n[1]; n[2] = -n[2]; d = -d;
                } else {
                    continue;
                }
                int dup = 0;
                for (int p = 0; p < np && !dup; ++p) {
                    const double* e = planes + 4 * p;
                    dup = n[0] * e[0] + n[1] * e[1] + n[2] * e[2] > 1.0 - 1e-12 && fabs(d - e[3]) <= eps;
                }
                if (dup) continue;
                if (np == max_planes) return -1;
                planes[4 * np] = n[0]; planes[4 * np + 1] = n[1]; planes[4 * np + 2] = n[2]; planes[4 * np + 3] = d;
                ++np;
            }
    return np >= 4 ? np : -1;
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

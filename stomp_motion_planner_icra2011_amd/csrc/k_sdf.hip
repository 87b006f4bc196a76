// k_sdf.hip -- the reference's distance-field fill on the device (StompCollisionSpace::setStartState,
// stomp_collision_space.cpp:154-197; paths relative to /root/reference/stomp_motion_planner/):
//   k_mark_lattice  one lane per lattice point of one object: environment boxes / cylinders
//                   sampled on the reference's running-sum lattice (addCollisionObjectsToPoints,
//                   :199-297; the per-axis coordinate lists are made on the host by the same loop),
//                   robot bodies (and meshes: their convex hull's planes) on the bounding-sphere
//                   lattice with a containment test (getVoxelsInBody, :592-650); the point goes
//                   through the object's frame and
//                   marks its cell (PropagationDistanceField::addPointsToField: round((p - o) / res)
//                   per axis, dropped unless inside the grid)
//   k_mark_points   the collision-map points (:205-211), marked the same way
//   k_edt_window    the capped exact EDT as three windowed minima (z from the marks, then y, then
//                   x), one lane per cell with the window along the axis; the lanes of a wave are
//                   consecutive z, so every window read is a coalesced row; the last pass writes
//                   min(d2, cap^2), the field's squared cell distance (distance = sqrt(d2) * res)
// oracle/sdf_oracle.c restates the same rules (with a sweep for the z pass); the tests compare the
// fields bit for bit.
#include <algorithm>

#include "kernels.h"

namespace stomp {

__device__ __forceinline__ bool mark_cell(const SdfMarkArgs& g, double px, double py, double pz)
{
    const double rx = round((px - g.o[0]) * g.inv_res);
    const double ry = round((py - g.o[1]) * g.inv_res);
    const double rz = round((pz - g.o[2]) * g.inv_res);
    if (!(rx >= 0.0 && rx < (double)g.n[0] && ry >= 0.0 && ry < (double)g.n[1] && rz >= 0.0 && rz < (double)g.n[2]))
        return false;
    const size_t idx = ((size_t)(long long)rx * g.n[1] + (size_t)(long long)ry) * g.n[2] + (size_t)(long long)rz;
    g.occ[idx] = 1;   // every writer stores 1
    return true;
}

__device__ __forceinline__ void count_marked(const SdfMarkArgs& g, bool hit)
{
    // every lane of the wave reaches this (no early exit in the marking kernels)
    const unsigned long long b = __ballot(hit);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(g.marked, (unsigned long long)__popcll(b));
}

__device__ __forceinline__ double dotcol(const double* v, const double* B, int k)
{
    return v[0] * B[k] + v[1] * B[3 + k] + v[2] * B[6 + k];
}

__global__ __launch_bounds__(256) void k_mark_lattice(SdfLatticeJob j, const double* axes, SdfMarkArgs g)
{
    const long long total = (long long)j.n[0] * j.n[1] * j.n[2];
    const long long idx = blockIdx.x * 256LL + threadIdx.x;
    bool hit = false;
    if (idx < total) {
        const int k = (int)(idx % j.n[2]);
        const int jj = (int)((idx / j.n[2]) % j.n[1]);
        const int i = (int)(idx / ((long long)j.n[2] * j.n[1]));
        const double* pos = j.pos;
        if (j.type == kShapeBox || j.type == kShapeCylinder) {
            const double x = axes[j.off[0] + i], y = axes[j.off[1] + jj], z = axes[j.off[2] + k];
            bool keep = true;
            if (j.type == kShapeCylinder) {   // :262-266
                const double xdist = fabs(pos[0] - x);
                const double ydist = fabs(pos[1] - y);
                keep = sqrt(xdist * xdist + ydist * ydist) <= j.dims[0];
            }
            if (keep) {
                const double p[3] = {pos[0] - x, pos[1] - y, pos[2] - z};
                double p2[3];
#pragma unroll
                for (int a = 0; a < 3; ++a)   // KDL Frame * Vector
                    p2[a] = j.R[3 * a + 0] * p[0] + j.R[3 * a + 1] * p[1] + j.R[3 * a + 2] * p[2] + pos[a];
                hit = mark_cell(g, p2[0], p2[1], p2[2]);
            }
        } else {
            // gridToWorld around the bounding-sphere centre (stomp_collision_space.h:237-241)
            const double w[3] = {(j.lo[0] + i) * j.res + pos[0], (j.lo[1] + jj) * j.res + pos[1],
                                 (j.lo[2] + k) * j.res + pos[2]};
            const double v[3] = {w[0] - pos[0], w[1] - pos[1], w[2] - pos[2]};
            const double* d = j.dims;
            bool in;
            if (j.type == kBodyMesh) {
                // bodies::ConvexMesh: inside every hull plane grown by the padding, in the body frame
                const double u[3] = {w[0] - j.org[0], w[1] - j.org[1], w[2] - j.org[2]};
                const double pb[3] = {dotcol(u, j.R, 0), dotcol(u, j.R, 1), dotcol(u, j.R, 2)};
                in = true;
                for (int q = 0; q < j.nplanes && in; ++q) {
                    const double* e = j.planes + 4 * q;
                    in = !(e[0] * pb[0] + e[1] * pb[1] + e[2] * pb[2] + e[3] > d[0]);
                }
            } else if (j.type == kBodySphere) {
                in = v[0] * v[0] + v[1] * v[1] + v[2] * v[2] < d[0] * d[0];
            } else if (j.type == kBodyBox) {
                in = !(fabs(dotcol(v, j.R, 0)) > d[0] / 2.0) && !(fabs(dotcol(v, j.R, 1)) > d[1] / 2.0) &&
                     !(fabs(dotcol(v, j.R, 2)) > d[2] / 2.0);
            } else {
                in = false;
                if (!(fabs(dotcol(v, j.R, 2)) > d[1] / 2.0)) {
                    const double b1 = dotcol(v, j.R, 0);
                    const double remaining = d[0] * d[0] - b1 * b1;
                    if (!(remaining < 0.0)) {
                        const double b2 = dotcol(v, j.R, 1);
                        in = b2 * b2 < remaining;
                    }
                }
            }
            if (in) hit = mark_cell(g, w[0], w[1], w[2]);
        }
    }
    count_marked(g, hit);
}

__global__ __launch_bounds__(256) void k_mark_points(const double* pts, long long np, SdfMarkArgs g)
{
    const long long i = blockIdx.x * 256LL + threadIdx.x;
    bool hit = false;
    if (i < np) hit = mark_cell(g, pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]);
    count_marked(g, hit);
}

// one windowed-minimum pass along `axis` (0 = x, 1 = y, 2 = z): out = min over |d| <= cap of
// in[cell + d] + d^2, kept <= far = cap^2 + 1 (any value above cap^2 means "beyond the cap").
// The z pass reads the marks (0 for a marked cell, far otherwise); the x pass writes the field.
template <int AXIS, bool FROM_OCC, bool FINAL>
__global__ __launch_bounds__(256) void k_edt_window(int nx, int ny, int nz, int cap, const void* in_raw,
                                                    unsigned short* out)
{
    const long long total = (long long)nx * ny * nz;
    const long long idx = blockIdx.x * 256LL + threadIdx.x;
    if (idx >= total) return;
    const int z = (int)(idx % nz);
    const int y = (int)((idx / nz) % ny);
    const int x = (int)(idx / ((long long)nz * ny));
    const int far = cap * cap + 1;
    const int c = AXIS == 0 ? x : (AXIS == 1 ? y : z);
    const int n = AXIS == 0 ? nx : (AXIS == 1 ? ny : nz);
    const long long stride = AXIS == 0 ? (long long)ny * nz : (AXIS == 1 ? nz : 1);
    const int lo = c - cap < 0 ? 0 : c - cap;
    const int hi = c + cap > n - 1 ? n - 1 : c + cap;
    const long long base = idx - (long long)c * stride;
    int best = far;
    if (FROM_OCC) {
        const unsigned char* occ = (const unsigned char*)in_raw;
        for (int q = lo; q <= hi; ++q) {
            const int d = q - c;
            const int v = occ[base + q * stride] ? d * d : far;
            best = v < best ? v : best;
        }
    } else {
        const unsigned short* a = (const unsigned short*)in_raw;
        for (int q = lo; q <= hi; ++q) {
            const int d = q - c;
            const int v = (int)a[base + q * stride] + d * d;
            best = v < best ? v : best;
        }
    }
    out[idx] = (unsigned short)(FINAL && best > far - 1 ? far - 1 : best);   // the last pass: min(d2, cap^2)
}

// [nx][ny][nz] -> 4^3 bricks (kernels.h DevModel::brick): one lane per destination voxel, so the
// stores are coalesced and each brick's 64 reads come from 16 z-runs of 4
__global__ __launch_bounds__(256) void k_sdf_bricks(const unsigned short* src, unsigned short* dst, int nx, int ny,
                                                    int nz, size_t total)
{
    const int nby = (ny + 3) / 4, nbz = (nz + 3) / 4;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const size_t b = i >> 6;
        const int in = (int)(i & 63);
        const int bz = (int)(b % nbz), by = (int)((b / nbz) % nby), bx = (int)(b / ((size_t)nbz * nby));
        const int x = 4 * bx + (in >> 4), y = 4 * by + ((in >> 2) & 3), z = 4 * bz + (in & 3);
        dst[i] = (x < nx && y < ny && z < nz) ? src[((size_t)x * ny + y) * nz + z] : (unsigned short)0;
    }
}

void launch_sdf_bricks(const unsigned short* src, unsigned short* dst, int nx, int ny, int nz, hipStream_t s)
{
    const size_t total = sdf_brick_cells(nx, ny, nz);
    const size_t blocks = std::min<size_t>((total + 255) / 256, 65536);
    hipLaunchKernelGGL(k_sdf_bricks, dim3((unsigned)blocks), dim3(256), 0, s, src, dst, nx, ny, nz, total);
}

void launch_mark_lattice(const SdfLatticeJob& j, const double* axes, const SdfMarkArgs& g, hipStream_t s)
{
    const long long total = (long long)j.n[0] * j.n[1] * j.n[2];
    if (total <= 0) return;
    hipLaunchKernelGGL(k_mark_lattice, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, j, axes, g);
}

void launch_mark_points(const double* pts, long long np, const SdfMarkArgs& g, hipStream_t s)
{
    if (np <= 0) return;
    hipLaunchKernelGGL(k_mark_points, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, s, pts, np, g);
}

void launch_edt(int nx, int ny, int nz, int cap, const unsigned char* occ, unsigned short* a, unsigned short* b,
                unsigned short* field, hipStream_t s)
{
    const long long total = (long long)nx * ny * nz;
    const dim3 grid((unsigned)((total + 255) / 256));
    hipLaunchKernelGGL((k_edt_window<2, true, false>), grid, dim3(256), 0, s, nx, ny, nz, cap, (const void*)occ, a);
    hipLaunchKernelGGL((k_edt_window<1, false, false>), grid, dim3(256), 0, s, nx, ny, nz, cap, (const void*)a, b);
    hipLaunchKernelGGL((k_edt_window<0, false, true>), grid, dim3(256), 0, s, nx, ny, nz, cap, (const void*)b, field);
}

}  // namespace stomp

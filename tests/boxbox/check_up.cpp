// box_box_deep_count_up (the upright specialisation used by k_tsp<..., UP>) against the generic
// box_box_deep_count on random upright box pairs: the deep-contact counts must be identical.
// Built and run by tests/test_boxbox_upright.py (host code, hipcc, -ffp-contract=off).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "sspp_device.h"

// the mover's rotation as mover_poses MODE 1 builds it (yaw_to_quat + normalize + quat2mat)
static void yaw_mat(double yaw, double* R) {
    const double half = yaw * 0.5;
    double w = cos(half), z = sin(half);
    const double nn = sqrt(fma(z, z, w * w));
    if (fabs(nn - 1.0) > sspd::kMinVal) { const double inv = 1.0 / nn; w *= inv; z *= inv; }
    const double q00 = w * w, q33 = z * z, q03 = w * z;
    R[0] = q00 - q33; R[1] = 2.0 * (0.0 - q03); R[2] = 0.0;
    R[3] = 2.0 * (0.0 + q03); R[4] = q00 - q33; R[5] = 0.0;
    R[6] = 0.0; R[7] = 0.0; R[8] = q00 + q33;
}

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 2000000;
    std::mt19937_64 rng(12345);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    long bad = 0, deep = 0, hist[9] = {0};
    const double yaws[] = {0.0, M_PI / 2, -M_PI / 2, M_PI, M_PI / 4, 1e-9};
    for (long it = 0; it < n; ++it) {
        double ma[9], mb[9], ea[3], eb[3], pa[3], pb[3];
        const int mode = (int)(it % 4);
        const double ya = (it % 7 == 0) ? 0.0 : (U(rng) - 0.5) * 7.0;
        const double yb = (it % 5 == 0) ? yaws[(it / 5) % 6] : (U(rng) - 0.5) * 7.0;
        if (it % 3 == 0) {  // identity static box (the stacking scene)
            for (int k = 0; k < 9; ++k) ma[k] = (k % 4 == 0) ? 1.0 : 0.0;
        } else {
            yaw_mat(ya, ma);
        }
        yaw_mat(yb, mb);
        if (it % 11 == 0) { for (int k : {1, 3, 4, 8}) mb[k] = -mb[k]; }  // z flipped (upright, mirrored)
        for (int k = 0; k < 3; ++k) {
            ea[k] = (it % 2 == 0) ? 0.1 : 0.02 + 0.1 * U(rng);
            eb[k] = (it % 2 == 0) ? 0.1 : 0.02 + 0.1 * U(rng);
            pa[k] = (U(rng) - 0.5) * 0.2;
        }
        // B near A: stacked on top, beside, or anywhere within reach
        const double s = ea[0] + ea[1] + eb[0] + eb[1];
        if (mode == 0) {
            pb[0] = pa[0] + (U(rng) - 0.5) * s; pb[1] = pa[1] + (U(rng) - 0.5) * s;
            pb[2] = pa[2] + ea[2] + eb[2] - 0.004 * U(rng);
        } else if (mode == 1) {
            pb[0] = pa[0] + (ea[0] + eb[0]) * (0.8 + 0.25 * U(rng)); pb[1] = pa[1] + (U(rng) - 0.5) * s;
            pb[2] = pa[2] + (U(rng) - 0.5) * 0.05;
        } else {
            for (int k = 0; k < 3; ++k) pb[k] = pa[k] + (U(rng) - 0.5) * 1.2 * (ea[k] + eb[k]) * 2;
        }
        const bool swap = it % 2 == 1;  // either box may be the first geom
        const int g = swap ? sspd::box_box_deep_count(pb, mb, eb, pa, ma, ea) : sspd::box_box_deep_count(pa, ma, ea, pb, mb, eb);
        const int u = swap ? sspd::box_box_deep_count_up(pb, mb, eb, pa, ma, ea) : sspd::box_box_deep_count_up(pa, ma, ea, pb, mb, eb);
        if (!sspd::upright3(ma) || !sspd::upright3(mb)) { printf("not upright\n"); return 2; }
        if (g != u) {
            if (bad < 5) printf("mismatch it=%ld generic=%d upright=%d\n", it, g, u);
            ++bad;
        }
        deep += g > 0;
        hist[g < 9 ? g : 8]++;
    }
    printf("pairs %ld deep %ld mismatches %ld counts", n, deep, bad);
    for (int k = 0; k < 9; ++k) printf(" %ld", hist[k]);
    printf("\n");
    return bad ? 1 : 0;
}

// Debug harness: the device EPnP (csrc/epnp.h) compiled for the host, to
// compare with the numpy oracle on CPU.  Not part of the product or tests.
#include "../orb-slam2-annotation_amd/csrc/epnp.h"

struct HostSrc {
    const float *P3, *P2;
    int n;
    int count() const { return n; }
    void get(int i, double* pw, double& u, double& v) const {
        pw[0] = P3[3 * i]; pw[1] = P3[3 * i + 1]; pw[2] = P3[3 * i + 2];
        u = P2[2 * i]; v = P2[2 * i + 1];
    }
};

extern "C" double epnp_host(int n, const float* P3, const float* P2, const double* cam, double* R, double* t) {
    HostSrc s{P3, P2, n};
    orbgpu::epnp::Pose p;
    const double e = orbgpu::epnp::compute_pose(s, orbgpu::epnp::Camera{cam[0], cam[1], cam[2], cam[3]}, p);
    for (int k = 0; k < 9; ++k) R[k] = p.R[k];
    for (int k = 0; k < 3; ++k) t[k] = p.t[k];
    return e;
}

extern "C" void eig_canon_host(const double* mtm_in, int k, double* ut) {
    double a[144], w[12];
    for (int i = 0; i < 144; ++i) a[i] = mtm_in[i];
    orbgpu::epnp::sym_eig_desc<12>(a, w, ut);
    if (k > 0) orbgpu::epnp::canonicalize_null_space(ut, k);
}

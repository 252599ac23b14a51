// On-device contact plans: gait template -> per-knot contact activation
// and foot poses for every problem of a batch, written straight into the handle's logic / pos /
// rot arrays, plus the reference's warm-start controls.
//
// Replaces the host preprocessing of create_contact_sequence / create_contact_trajectory
// (reference src/contact_plan.py:40-48, 112-264) and Centroidal_model.__fill_contact_data /
// __fill_initial_trajectory (src/centroidal_model.py:127-187).  The plan of one problem is a
// closed-form function of the knot index: phases repeat as [support, step A, support, step B]
// (one extra support phase after the last step), swing feet are inactive, stance feet sit at
// their initial position advanced by stepLength once per completed step of their set.  The
// advance is accumulated by repeated addition, exactly as the reference's `+=` per phase, so
// the positions are bit-identical to the host construction.  Rotations are angle-axis
// (angle = 0, src/contact_plan.py:166): the identity.  One thread per (problem, knot).
#include "common.hpp"

namespace cmpc {

// swing sets (bit c = contact c in the order FR, FL, HR, HL / FR, FL) of the two step phases
template <int ROBOT> __device__ __forceinline__ void step_sets(int type, unsigned &a, unsigned &b) {
    if (ROBOT == 0) {
        if (type == CMPC_GAIT_TROT) { a = 0x9u; b = 0x6u; }          // rflhStep {FR, HL} | lfrhStep {FL, HR}
        else if (type == CMPC_GAIT_PACE) { a = 0x5u; b = 0xAu; }     // rfrhStep {FR, HR} | lflhStep {FL, HL}
        else { a = 0x3u; b = 0xCu; }                                 // rflfStep {FR, FL} | rhlhStep {HR, HL}
    } else {
        if (type == CMPC_GAIT_PACE) { a = 0x1u; b = 0x2u; }          // rfStep {FR} | lfStep {FL}
        else { a = 0x3u; b = 0x3u; }   // TALOS has no trot / bound phases: the reference's
                                       // fall-through swings and advances every foot (:254-263)
    }
}

template <typename T, int ROBOT>
__global__ void __launch_bounds__(128) k_contact_plan(DevBuf<T> d, const cmpc_gait *gaits, const T *foot0,
                                                      uint8_t *logic, T *pos, T *rot) {
    constexpr int NC = Robot<ROBOT>::NC;
    const int N = d.N;
    const long g = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= (long)d.B * N) return;
    const int b = (int)(g / N), k = (int)(g % N);
    const cmpc_gait gt = gaits[b];
    const int sup = gt.support_knots, stp = gt.step_knots, cyc = 2 * (sup + stp);
    const int s = k / cyc, r = k % cyc;
    unsigned A, Bs;
    step_sets<ROBOT>(gt.type, A, Bs);
    // swing set of the current phase and the step phases completed before knot k
    unsigned swing = 0u;
    if (s < gt.nb_steps) {
        if (r >= sup && r < sup + stp) swing = A;
        else if (r >= 2 * sup + stp) swing = Bs;
    }
    const int nA = s + (s < gt.nb_steps && r >= sup + stp ? 1 : 0), nB = s;
    const T L = T(gt.step_length);
    for (int c = 0; c < NC; ++c) {
        const bool act = !((swing >> c) & 1u);
        const int adv = (((A >> c) & 1u) ? nA : 0) + (((Bs >> c) & 1u) ? nB : 0);
        const T *f0 = foot0 + ((size_t)b * NC + c) * 3;
        T x = f0[0];
        for (int i = 0; i < adv; ++i) x += L;   // feet[c][0] += stepLength after each of its steps
        const size_t o = (size_t)g * NC + c;
        logic[o] = act ? 1 : 0;
        pos[o * 3 + 0] = act ? x : T(0);
        pos[o * 3 + 1] = act ? f0[1] : T(0);
        pos[o * 3 + 2] = act ? f0[2] : T(0);
        for (int e = 0; e < 9; ++e) rot[o * 9 + e] = act ? ((e % 4 == 0) ? T(1) : T(0)) : T(0);
    }
}

// warm-start controls (src/centroidal_model.py:176-183): per active contact i, rows 3i..3i+2 =
// [1e-3, 1e-3, m * 9.81 / #active] (3i also for TALOS, quirk Q11); zero elsewhere
template <typename T, int ROBOT> __global__ void __launch_bounds__(128) k_default_controls(DevBuf<T> d, T *Ubar) {
    constexpr int NC = Robot<ROBOT>::NC;
    const int N = d.N;
    const long g = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= (long)d.B * N) return;
    const int b = (int)(g / N);
    const DevParams<T> &prm = d.params[d.class_id[b]];
    const uint8_t *lg = d.logic + (size_t)g * NC;
    int nact = 0;
    for (int c = 0; c < NC; ++c) nact += lg[c] ? 1 : 0;
    T *u = Ubar + (size_t)g * NU;
    for (int i = 0; i < NU; ++i) u[i] = T(0);
    const T fz = (-prm.mass * prm.gravity) / T(nact);   // robot_weight = -m g (:176)
    for (int c = 0; c < NC; ++c)
        if (lg[c]) { u[3 * c] = T(1e-3); u[3 * c + 1] = T(1e-3); u[3 * c + 2] = fz; }
}

#define INST(T, R)                                                                                           \
    template __global__ void k_contact_plan<T, R>(DevBuf<T>, const cmpc_gait *, const T *, uint8_t *, T *, T *); \
    template __global__ void k_default_controls<T, R>(DevBuf<T>, T *);
INST(double, 0)
INST(double, 1)
INST(float, 0)
INST(float, 1)
#undef INST

}  // namespace cmpc

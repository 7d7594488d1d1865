/*
 * oracle.c -- fp64 CPU restatement of the reference's physics step (TEST
 * INFRASTRUCTURE ONLY; see oracle.h for who may load it).
 *
 * Reference call chain restated here:
 *   GazeboRuntime.step            python/gym_ignition/runtimes/gazebo_runtime.py:91-120
 *   Physics::Update               cpp/scenario/plugins/Physics/Physics.cpp:646-685
 *     UpdatePhysics (resets/cmds) Physics.cpp:1330-1440 (velocity reset, then
 *                                 position reset, then SetForce per dof)
 *     Step -> dartsim ForwardStep Physics.cpp:1824-1835  [EXT: DART 6.x World::step]
 *     UpdateSim readback          Physics.cpp:2250-2254 (zero JointForceCmd),
 *                                 :2276-2345 (position/velocity/acceleration/force)
 *
 * DART 6.x World::step [EXT, restated from its published algorithm]:
 *   computeForwardDynamics   articulated-body algorithm; the projected
 *                            articulated inertia carries the implicit damping
 *                            term S^T AI S + dt*d (GenericJoint::
 *                            updateInvProjArtInertiaImplicit) and the joint
 *                            force is tau - d*qd - S^T(AI eta + B)
 *                            (GenericJoint::updateTotalForceDynamic)
 *   integrateVelocities      qd += dt * qdd
 *   ConstraintSolver::solve  joint-limit / servo / Coulomb-friction rows
 *                            (JointLimitConstraint, ServoMotorConstraint,
 *                            JointCoulombFrictionConstraint) as a boxed LCP
 *                            A x = b + w with A = J M^-1 J^T (CFM 1e-9)
 *   computeImpulseForwardDynamics  dqd = M^-1 J^T x (non-implicit AI)
 *   integratePositions       q += dt * qd
 * Force commands are clipped to +-effort (GenericJoint::setCommand, FORCE).
 *
 * Spatial conventions (DART): spatial vectors are [angular; linear] in body
 * coordinates; T = (R, p) is the child pose in the parent; X = Ad_{T^-1}.
 */
#include "oracle.h"

#include <math.h>
#include <string.h>

/* Ground-contact slots of a collision shape (Physics.cpp:687-1219 builds box,
 * sphere and cylinder collisions; the kernels' twin is chain_dyn.hpp
 * shape_slot_point): the shape-frame point of slot c.  Box (h = half
 * extents): corner c (bits x y z); sphere: its centre (lowered by the radius by
 * the caller); cylinder (h = {radius, half length}, axis z): 4 rim points per
 * cap (c & 4: the +z cap), 90 degrees apart from the rim point deepest along
 * the plane normal.  RS = the shape's world rotation (Rb SR). */
void or_slot_point(int type, const double* h, const double* RS, int c, double l[3])
{
    l[0] = l[1] = l[2] = 0.0;
    if (type == 0) {
        l[0] = (c & 4) ? h[0] : -h[0];
        l[1] = (c & 2) ? h[1] : -h[1];
        l[2] = (c & 1) ? h[2] : -h[2];
    } else if (type == 2) {
        double ux = -RS[6], uy = -RS[7];   /* -(world z in the shape frame), projected on the cap plane */
        const double n2 = ux * ux + uy * uy;
        if (n2 > 1e-12) {
            const double inv = 1.0 / sqrt(n2);
            ux *= inv;
            uy *= inv;
        } else {
            ux = 1.0;
            uy = 0.0;
        }
        const int j = c & 3;
        const double dx = (j == 0) ? ux : ((j == 1) ? -uy : ((j == 2) ? -ux : uy));
        const double dy = (j == 0) ? uy : ((j == 1) ? ux : ((j == 2) ? -uy : -ux));
        l[0] = h[0] * dx;
        l[1] = h[0] * dy;
        l[2] = (c & 4) ? h[1] : -h[1];
    }
}

static void rot_mul(const double* A, const double* B, double* C)
{
    for (int r = 0; r < 3; ++r)
        for (int k = 0; k < 3; ++k) C[r * 3 + k] = A[r * 3] * B[k] + A[r * 3 + 1] * B[3 + k] + A[r * 3 + 2] * B[6 + k];
}


/* ---------------- small dense helpers (6x6 row-major) ---------------- */

static void m6_zero(double* A) { memset(A, 0, 36 * sizeof(double)); }

static void m6_vec(const double* A, const double* x, double* y)
{
    for (int i = 0; i < 6; ++i) {
        double s = 0.0;
        for (int k = 0; k < 6; ++k) s += A[i * 6 + k] * x[k];
        y[i] = s;
    }
}

static void m6t_vec(const double* A, const double* x, double* y)
{
    for (int i = 0; i < 6; ++i) {
        double s = 0.0;
        for (int k = 0; k < 6; ++k) s += A[k * 6 + i] * x[k];
        y[i] = s;
    }
}

/* out = X^T I X */
static void m6_congruence(const double* X, const double* I, double* out)
{
    double T[36];
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
            double s = 0.0;
            for (int k = 0; k < 6; ++k) s += I[i * 6 + k] * X[k * 6 + j];
            T[i * 6 + j] = s;
        }
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
            double s = 0.0;
            for (int k = 0; k < 6; ++k) s += X[k * 6 + i] * T[k * 6 + j];
            out[i * 6 + j] = s;
        }
}

static double dot6(const double* a, const double* b)
{
    double s = 0.0;
    for (int i = 0; i < 6; ++i) s += a[i] * b[i];
    return s;
}

static void cross3(const double* a, const double* b, double* c)
{
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

/* ad(V) W = [w x a ; w x b + v x a] */
static void sp_ad(const double* V, const double* W, double* out)
{
    double t[3];
    cross3(V, W, out);
    cross3(V, W + 3, out + 3);
    cross3(V + 3, W, t);
    out[3] += t[0]; out[4] += t[1]; out[5] += t[2];
}

/* dad(V, F) = ad(V)^T F = [n x w + f x v ; f x w] */
static void sp_dad(const double* V, const double* F, double* out)
{
    double t[3];
    cross3(F, V, out);
    cross3(F + 3, V + 3, t);
    out[0] += t[0]; out[1] += t[1]; out[2] += t[2];
    cross3(F + 3, V, out + 3);
}

/* ---------------- model kinematics / inertia ---------------- */

/* DART's BallJoint (a MultiDofJoint<3>; Joint.cpp:267-331 exposes it as
 * core::JointType::Ball): positions = the rotation vector theta of the joint
 * rotation, velocities = the child's angular velocity in its own frame, the
 * relative Jacobian [I; 0] constant, positions integrated on SO(3) as
 * R <- R exp(dt w) [EXT: dart/dynamics/BallJoint.cpp].  The model lists it as
 * three bodies at one point (jtype bits 4-5 = part 1, 2, 3; unit axes x, y, z;
 * the first two massless): part 1 carries the whole rotation E exp(theta),
 * theta = (q_i, q_i+1, q_i+2), parts 2 and 3 have identity transforms, so the
 * three motion axes are the child frame's and qd of the parts is w. */
static int ball_part(const or_model* m, int i) { return (m->jtype[i] >> 4) & 3; }

/* exp of a rotation vector (Rodrigues) */
static void so3_exp(const double th[3], double R[9])
{
    const double t2 = th[0] * th[0] + th[1] * th[1] + th[2] * th[2], t = sqrt(t2);
    const double A = (t < 1e-8) ? 1.0 - t2 / 6.0 : sin(t) / t;
    const double B = (t < 1e-8) ? 0.5 - t2 / 24.0 : (1.0 - cos(t)) / t2;
    const double K[9] = {0, -th[2], th[1], th[2], 0, -th[0], -th[1], th[0], 0};
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            double kk = 0.0;
            for (int j = 0; j < 3; ++j) kk += K[r * 3 + j] * K[j * 3 + c];
            R[r * 3 + c] = (r == c ? 1.0 : 0.0) + A * K[r * 3 + c] + B * kk;
        }
}

/* unit quaternion (w, x, y, z) of a rotation vector, and back (angle in [0, pi]) */
static void rotvec_quat(const double th[3], double qt[4])
{
    const double t = sqrt(th[0] * th[0] + th[1] * th[1] + th[2] * th[2]);
    const double s = (t < 1e-8) ? 0.5 - t * t / 48.0 : sin(0.5 * t) / t;
    qt[0] = cos(0.5 * t); qt[1] = s * th[0]; qt[2] = s * th[1]; qt[3] = s * th[2];
}
static void quat_rotvec(const double qt[4], double th[3])
{
    double w = qt[0], x = qt[1], y = qt[2], z = qt[3];
    if (w < 0.0) { w = -w; x = -x; y = -y; z = -z; }
    const double v = sqrt(x * x + y * y + z * z);
    const double k = (v < 1e-12) ? 2.0 / w : 2.0 * atan2(v, w) / v;
    th[0] = k * x; th[1] = k * y; th[2] = k * z;
}

/* BallJoint::integratePositions: theta <- log(exp(theta) exp(dt w)) */
static void ball_integrate(double th[3], const double w[3], double dt)
{
    double a[4], b[4], c[4];
    const double dw[3] = {dt * w[0], dt * w[1], dt * w[2]};
    rotvec_quat(th, a);
    rotvec_quat(dw, b);
    c[0] = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
    c[1] = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
    c[2] = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
    c[3] = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
    quat_rotvec(c, th);
}

/* integratePositions of the tree's joints: q += dt qd, a ball joint on SO(3) */
static void integrate_joint_positions(const or_model* m, double* q, const double* qd, double dt)
{
    for (int i = 0; i < m->n; ++i) {
        const int bp = ball_part(m, i);
        if (bp == 1) {
            ball_integrate(q + i, qd + i, dt);
            i += 2;
        } else if (bp == 0) {
            q[i] += dt * qd[i];
        }
    }
}

/* ad(V, S qd) of joint i (the velocity-product acceleration); a ball joint's
 * parts 2 and 3 see V without the ball's earlier parts (one joint of
 * constant S: the ball's own S qd x S qd vanishes) */
static void joint_bias(const or_model* m, int i, const double* qd, const double V[6], const double Sq[6], double out[6])
{
    const int bp = ball_part(m, i);
    double Ve[6];
    memcpy(Ve, V, sizeof Ve);
    if (bp >= 2) Ve[0] -= qd[i - bp + 1];
    if (bp == 3) Ve[1] -= qd[i - 1];
    sp_ad(Ve, Sq, out);
}

static void joint_pose(const or_model* m, int i, const double* qv, double R[9], double p[3])
{
    const double* E = m->E[i];
    const double* a = m->axis[i];
    const int bp = ball_part(m, i);
    if (bp) {
        double X[9];
        if (bp == 1) so3_exp(qv + i, X);
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c)
                R[r * 3 + c] = (bp == 1) ? E[r * 3] * X[c] + E[r * 3 + 1] * X[3 + c] + E[r * 3 + 2] * X[6 + c]
                                         : E[r * 3 + c];
        p[0] = m->r[i][0]; p[1] = m->r[i][1]; p[2] = m->r[i][2];
        return;
    }
    const double q = qv[i];
    if ((m->jtype[i] & 1) == 0) {
        const double c = cos(q), s = sin(q), v = 1.0 - c;
        double J[9];
        J[0] = c + a[0] * a[0] * v;        J[1] = a[0] * a[1] * v - a[2] * s; J[2] = a[0] * a[2] * v + a[1] * s;
        J[3] = a[1] * a[0] * v + a[2] * s; J[4] = c + a[1] * a[1] * v;        J[5] = a[1] * a[2] * v - a[0] * s;
        J[6] = a[2] * a[0] * v - a[1] * s; J[7] = a[2] * a[1] * v + a[0] * s; J[8] = c + a[2] * a[2] * v;
        for (int r = 0; r < 3; ++r)
            for (int cidx = 0; cidx < 3; ++cidx)
                R[r * 3 + cidx] = E[r * 3] * J[cidx] + E[r * 3 + 1] * J[3 + cidx] + E[r * 3 + 2] * J[6 + cidx];
        p[0] = m->r[i][0]; p[1] = m->r[i][1]; p[2] = m->r[i][2];
    } else {
        memcpy(R, E, 9 * sizeof(double));
        for (int r = 0; r < 3; ++r)
            p[r] = m->r[i][r] + q * (E[r * 3] * a[0] + E[r * 3 + 1] * a[1] + E[r * 3 + 2] * a[2]);
    }
}

/* X = Ad_{T^-1} = [[R^T, 0], [-R^T [p]x, R^T]] */
static void plucker(const double R[9], const double p[3], double X[36])
{
    m6_zero(X);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            X[r * 6 + c] = R[c * 3 + r];
            X[(r + 3) * 6 + c + 3] = R[c * 3 + r];
        }
    const double P[9] = {0, -p[2], p[1], p[2], 0, -p[0], -p[1], p[0], 0};
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            double s = 0.0;
            for (int k = 0; k < 3; ++k) s += R[k * 3 + r] * P[k * 3 + c];
            X[(r + 3) * 6 + c] = -s;
        }
}

static void motion_subspace(const or_model* m, int i, double S[6])
{
    memset(S, 0, 6 * sizeof(double));
    const int off = ((m->jtype[i] & 1) == 0) ? 0 : 3;
    S[off] = m->axis[i][0]; S[off + 1] = m->axis[i][1]; S[off + 2] = m->axis[i][2];
}

/* spatial inertia about the body origin, [angular; linear] ordering */
static void body_inertia(const or_model* m, int i, double I[36])
{
    const double ms = m->mass[i];
    const double* c = m->com[i];
    const double* ic = m->Ic[i];
    const double Icm[9] = {ic[0], ic[3], ic[4], ic[3], ic[1], ic[5], ic[4], ic[5], ic[2]};
    const double C[9] = {0, -c[2], c[1], c[2], 0, -c[0], -c[1], c[0], 0};
    m6_zero(I);
    for (int r = 0; r < 3; ++r)
        for (int k = 0; k < 3; ++k) {
            double cc = 0.0; /* -[c]x[c]x */
            for (int j = 0; j < 3; ++j) cc -= C[r * 3 + j] * C[j * 3 + k];
            I[r * 6 + k] = Icm[r * 3 + k] + ms * cc;
            I[r * 6 + k + 3] = ms * C[r * 3 + k];
            I[(r + 3) * 6 + k] = -ms * C[r * 3 + k];
            I[(r + 3) * 6 + k + 3] = (r == k) ? ms : 0.0;
        }
}

/* ---------------- articulated-body algorithm ---------------- */

typedef struct {
    double X[OR_MAXB][36];
    double S[OR_MAXB][6];
    double U[OR_MAXB][6];    /* AI S (non-implicit)      */
    double Psi[OR_MAXB];     /* (S^T AI S)^-1             */
} or_impulse_factor;

/* Tree ABA (Featherstone 2008, Table 7.1) with DART's implicit damping.
 * Bodies are in depth-first order (parent[i] < i), so the outward passes run
 * i = 0..n-1 and the inward pass i = n-1..0 accumulates into parent[i]. */
static void aba_full(const or_model* m, const double* q, const double* qd,
                     const double* tau, double dt_implicit, double* qdd,
                     or_impulse_factor* fac)
{
    const int n = m->n;
    double X[OR_MAXB][36], S[OR_MAXB][6], eta[OR_MAXB][6], B[OR_MAXB][6];
    double I[OR_MAXB][36], AIi[OR_MAXB][36], AI[OR_MAXB][36];
    double Ui[OR_MAXB][6], Psii[OR_MAXB], tt[OR_MAXB];
    double V[OR_MAXB][6], g[OR_MAXB][3];

    for (int i = 0; i < n; ++i) {
        double R[9], p[3], Vp[6], Sq[6], IV[6], dd[6], Fg[6], ga[6] = {0};
        const int pa = m->parent[i];
        const double zero6[6] = {0}, *Vpar = pa < 0 ? zero6 : V[pa];
        const double* gpar = pa < 0 ? m->gravity_base : g[pa];
        joint_pose(m, i, q, R, p);
        plucker(R, p, X[i]);
        motion_subspace(m, i, S[i]);
        m6_vec(X[i], Vpar, Vp);
        for (int k = 0; k < 6; ++k) { Sq[k] = S[i][k] * qd[i]; V[i][k] = Vp[k] + Sq[k]; }
        for (int r = 0; r < 3; ++r) g[i][r] = R[r] * gpar[0] + R[3 + r] * gpar[1] + R[6 + r] * gpar[2];
        joint_bias(m, i, qd, V[i], Sq, eta[i]);
        body_inertia(m, i, I[i]);
        m6_vec(I[i], V[i], IV);
        sp_dad(V[i], IV, dd);
        ga[3] = g[i][0]; ga[4] = g[i][1]; ga[5] = g[i][2];
        m6_vec(I[i], ga, Fg);
        for (int k = 0; k < 6; ++k) B[i][k] = -dd[k] - Fg[k];
        memcpy(AIi[i], I[i], sizeof(double) * 36);
        memcpy(AI[i], I[i], sizeof(double) * 36);
    }

    for (int i = n - 1; i >= 0; --i) {
        double U[6], AIeta[6], tmp[6];
        const int pa = m->parent[i];
        m6_vec(AIi[i], S[i], Ui[i]);
        Psii[i] = 1.0 / (dot6(S[i], Ui[i]) + dt_implicit * m->damping[i]);
        m6_vec(AI[i], S[i], U);
        const double psi = 1.0 / dot6(S[i], U);
        if (fac) { memcpy(fac->U[i], U, sizeof U); fac->Psi[i] = psi; }
        m6_vec(AIi[i], eta[i], AIeta);
        for (int k = 0; k < 6; ++k) tmp[k] = AIeta[k] + B[i][k];
        tt[i] = tau[i] - m->damping[i] * qd[i] - dot6(S[i], tmp);
        if (pa >= 0) {
            double Pi[36], Pn[36], beta[6], c[36], bp[6];
            for (int r = 0; r < 6; ++r)
                for (int k = 0; k < 6; ++k) {
                    Pi[r * 6 + k] = AIi[i][r * 6 + k] - Psii[i] * Ui[i][r] * Ui[i][k];
                    Pn[r * 6 + k] = AI[i][r * 6 + k] - psi * U[r] * U[k];
                }
            for (int k = 0; k < 6; ++k) beta[k] = B[i][k] + AIeta[k] + Ui[i][k] * Psii[i] * tt[i];
            m6_congruence(X[i], Pi, c);
            for (int k = 0; k < 36; ++k) AIi[pa][k] += c[k];
            m6_congruence(X[i], Pn, c);
            for (int k = 0; k < 36; ++k) AI[pa][k] += c[k];
            m6t_vec(X[i], beta, bp);
            for (int k = 0; k < 6; ++k) B[pa][k] += bp[k];
        }
    }

    double a[OR_MAXB][6];
    for (int i = 0; i < n; ++i) {
        double ap[6];
        const int pa = m->parent[i];
        const double zero6[6] = {0};
        m6_vec(X[i], pa < 0 ? zero6 : a[pa], ap);
        qdd[i] = Psii[i] * (tt[i] - dot6(Ui[i], ap));
        for (int k = 0; k < 6; ++k) a[i][k] = ap[k] + eta[i][k] + S[i][k] * qdd[i];
    }
    if (fac) {
        for (int i = 0; i < n; ++i) {
            memcpy(fac->X[i], X[i], sizeof(double) * 36);
            memcpy(fac->S[i], S[i], sizeof(double) * 6);
        }
    }
}

void or_aba(const or_model* m, const double* q, const double* qd,
            const double* tau, double dt_implicit, double* qdd)
{
    aba_full(m, q, qd, tau, dt_implicit, qdd, 0);
}

/* velocity change of every dof for a unit generalized impulse on dof j
 * (DART computeImpulseForwardDynamics with only joint impulses): the bias
 * impulse is nonzero only on the ancestors of j; the outward pass reaches
 * every body. */
static void impulse_column(const or_model* m, const or_impulse_factor* f, int j,
                           double* col)
{
    const int n = m->n;
    double u[OR_MAXB], Bimp[OR_MAXB][6];
    memset(Bimp, 0, sizeof(double) * 6 * (size_t)n);
    for (int i = n - 1; i >= 0; --i) {
        u[i] = (i == j ? 1.0 : 0.0) - dot6(f->S[i], Bimp[i]);
        const int pa = m->parent[i];
        if (pa >= 0) {
            double t[6], bp[6];
            for (int k = 0; k < 6; ++k) t[k] = Bimp[i][k] + f->U[i][k] * f->Psi[i] * u[i];
            m6t_vec(f->X[i], t, bp);
            for (int k = 0; k < 6; ++k) Bimp[pa][k] += bp[k];
        }
    }
    double dv[OR_MAXB][6];
    for (int i = 0; i < n; ++i) {
        double dvp[6];
        const int pa = m->parent[i];
        const double zero6[6] = {0};
        m6_vec(f->X[i], pa < 0 ? zero6 : dv[pa], dvp);
        col[i] = f->Psi[i] * (u[i] - dot6(f->U[i], dvp));
        for (int k = 0; k < 6; ++k) dv[i][k] = dvp[k] + f->S[i][k] * col[i];
    }
}

void or_crba(const or_model* m, const double* q, double* M)
{
    const int n = m->n;
    double X[OR_MAXB][36], S[OR_MAXB][6], Ic[OR_MAXB][36];
    for (int i = 0; i < n; ++i) {
        double R[9], p[3];
        joint_pose(m, i, q, R, p);
        plucker(R, p, X[i]);
        motion_subspace(m, i, S[i]);
        body_inertia(m, i, Ic[i]);
    }
    for (int i = n - 1; i >= 0; --i) {
        const int pa = m->parent[i];
        if (pa < 0) continue;
        double c[36];
        m6_congruence(X[i], Ic[i], c);
        for (int k = 0; k < 36; ++k) Ic[pa][k] += c[k];
    }
    for (int i = 0; i < n * n; ++i) M[i] = 0.0;
    for (int i = 0; i < n; ++i) {
        double F[6];
        m6_vec(Ic[i], S[i], F);
        M[i * n + i] = dot6(S[i], F);
        for (int j = i; m->parent[j] >= 0;) {
            double Fp[6];
            m6t_vec(X[j], F, Fp);
            memcpy(F, Fp, sizeof F);
            j = m->parent[j];
            M[i * n + j] = dot6(S[j], F);
            M[j * n + i] = M[i * n + j];
        }
    }
}

void or_rnea(const or_model* m, const double* q, const double* qd,
             const double* qdd, double* tau)
{
    const int n = m->n;
    double X[OR_MAXB][36], S[OR_MAXB][6], f[OR_MAXB][6];
    double V[OR_MAXB][6], a[OR_MAXB][6];
    const double V0[6] = {0};
    const double a0[6] = {0, 0, 0, -m->gravity_base[0], -m->gravity_base[1], -m->gravity_base[2]};
    for (int i = 0; i < n; ++i) {
        double R[9], p[3], Vp[6], ap[6], Sq[6], c[6], I[36], Ia[6], IV[6], dd[6];
        const int pa = m->parent[i];
        joint_pose(m, i, q, R, p);
        plucker(R, p, X[i]);
        motion_subspace(m, i, S[i]);
        m6_vec(X[i], pa < 0 ? V0 : V[pa], Vp);
        m6_vec(X[i], pa < 0 ? a0 : a[pa], ap);
        for (int k = 0; k < 6; ++k) { Sq[k] = S[i][k] * qd[i]; V[i][k] = Vp[k] + Sq[k]; }
        joint_bias(m, i, qd, V[i], Sq, c);
        for (int k = 0; k < 6; ++k) a[i][k] = ap[k] + S[i][k] * qdd[i] + c[k];
        body_inertia(m, i, I);
        m6_vec(I, a[i], Ia);
        m6_vec(I, V[i], IV);
        sp_dad(V[i], IV, dd);
        for (int k = 0; k < 6; ++k) f[i][k] = Ia[k] - dd[k];
    }
    for (int i = n - 1; i >= 0; --i) {
        tau[i] = dot6(S[i], f[i]);
        const int pa = m->parent[i];
        if (pa >= 0) {
            double fp[6];
            m6t_vec(X[i], f[i], fp);
            for (int k = 0; k < 6; ++k) f[pa][k] += fp[k];
        }
    }
}

/* ---------------- boxed LCP ---------------- */

/* Sweep budget: iters >= 0 runs exactly that many Gauss-Seidel sweeps (the
 * GPU kernels' PGS-only mode).  iters < 0 (OR_PGS_CONVERGED) solves the boxed
 * LCP the way DART does (lcp_dantzig below: ODE's Dantzig solver with its
 * friction index, two strictly convex box QPs solved exactly), after
 * OR_PGS_WARM sweeps that only pick the starting point.  or_pgs_stats():
 * sweeps (+ 1e6 x box-QP iterations) of the latest solve and its final
 * complementarity residual. */
#define OR_PGS_WARM 300
#define OR_LCP_MAXN0 (3 * OR_MAXFC + 3 * OR_MAXB > 3 * OR_MAXCONTACTS ? 3 * OR_MAXFC + 3 * OR_MAXB : 3 * OR_MAXCONTACTS)
/* ... and the scene step's rows (3 OR_SC_MAXC contact rows + joint rows) */
#define OR_LCP_MAXN (OR_LCP_MAXN0 > 3 * OR_SC_MAXC + 3 * OR_MAXB ? OR_LCP_MAXN0 : 3 * OR_SC_MAXC + 3 * OR_MAXB)
static _Thread_local int g_pgs_sweeps = 0;
static _Thread_local double g_pgs_delta = 0.0;

void or_pgs_stats(int* sweeps, double* last_delta)
{
    if (sweeps) *sweeps = g_pgs_sweeps;
    if (last_delta) *last_delta = g_pgs_delta;
}

/* Test hook: a copy of the latest floating-tree LCP (rows, Delassus matrix
 * with CFM, rhs, bounds, row kinds 0 normal / 1 friction / 2 box, the friction
 * coefficient) and the impulses the solve returned -- lets tests/ replay the
 * exact problem the kernels solve (tests/test_lcp_exact.py). */
#define OR_CAP_MAXN (3 * OR_MAXFC + 3 * OR_MAXB)
static _Thread_local double g_cap_A[OR_CAP_MAXN * OR_CAP_MAXN], g_cap_b[OR_CAP_MAXN], g_cap_lo[OR_CAP_MAXN],
    g_cap_hi[OR_CAP_MAXN], g_cap_x[OR_CAP_MAXN], g_cap_mu;
static _Thread_local int g_cap_kind[OR_CAP_MAXN], g_cap_n = 0;
/* row identities of the capture (the kernels' warm-record index: contact slot
 * rows 3 slot + d, joint rows OR_WARM_JOINT0 + 3 dof + type; -1 where the
 * step has none, e.g. the scene step) and DART's stage-1 impulses of the
 * converged mode (lcp_dantzig: friction rows 0) */
static _Thread_local int g_cap_wid[OR_CAP_MAXN];
static _Thread_local double g_cap_x1[OR_CAP_MAXN];
/* per row, the magnitude of the terms b_r is formed from (sum_e |J_re nu_e|
 * plus the bias velocity): the scale of b's rounding error in a finite
 * precision step (tests/lcp_validity.py) */
static _Thread_local double g_cap_bscale[OR_CAP_MAXN];
static _Thread_local double g_last_x1[OR_CAP_MAXN + 64];

int or_lcp_last(int cap, double* A, double* b, double* lo, double* hi, int* kind, double* x, double* mu)
{
    const int n = g_cap_n;
    if (n > cap) return -n;
    for (int r = 0; r < n; ++r) {
        for (int c = 0; c < n; ++c) A[r * n + c] = g_cap_A[r * n + c];
        b[r] = g_cap_b[r]; lo[r] = g_cap_lo[r]; hi[r] = g_cap_hi[r]; kind[r] = g_cap_kind[r]; x[r] = g_cap_x[r];
    }
    *mu = g_cap_mu;
    return n;
}

int or_lcp_last_rows(int cap, int32_t* wid, double* x1, double* bscale)
{
    const int n = g_cap_n;
    if (n > cap) return -n;
    for (int r = 0; r < n; ++r) {
        wid[r] = g_cap_wid[r];
        x1[r] = g_cap_x1[r];
        bscale[r] = g_cap_bscale[r];
    }
    return n;
}

static int pgs_budget(int iters) { return iters >= 0 ? iters : OR_PGS_WARM; }

static void pgs_count(int it) { g_pgs_sweeps = it + 1; g_pgs_delta = 0.0; }

/* bounds of row r at impulses x: findex[r] >= 0 marks a friction row whose
 * box is [-mu x_f, mu x_f] (x_f: its contact's normal impulse) */
static void row_bounds(int r, const double* lo, const double* hi, const int* findex, double mu,
                       const double* x, double* L, double* U)
{
    if (findex[r] >= 0) {
        const double u = mu * x[findex[r]];
        *L = -u;
        *U = u;
    } else {
        *L = lo[r];
        *U = hi[r];
    }
}

/* dense Gaussian elimination with partial pivoting, n <= OR_LCP_MAXN; 0 if singular */
static int lcp_gauss(int n, double* K, double* c, double* y)
{
    for (int col = 0; col < n; ++col) {
        int piv = col;
        for (int r = col + 1; r < n; ++r)
            if (fabs(K[r * n + col]) > fabs(K[piv * n + col])) piv = r;
        if (K[piv * n + col] == 0.0) return 0;
        if (piv != col) {
            for (int e = 0; e < n; ++e) { double t = K[col * n + e]; K[col * n + e] = K[piv * n + e]; K[piv * n + e] = t; }
            double t = c[col]; c[col] = c[piv]; c[piv] = t;
        }
        for (int r = col + 1; r < n; ++r) {
            const double f = K[r * n + col] / K[col * n + col];
            if (f == 0.0) continue;
            for (int e = col; e < n; ++e) K[r * n + e] -= f * K[col * n + e];
            c[r] -= f * c[col];
        }
    }
    for (int r = n - 1; r >= 0; --r) {
        double acc = c[r];
        for (int e = r + 1; e < n; ++e) acc -= K[r * n + e] * y[e];
        y[r] = acc / K[r * n + r];
    }
    return 1;
}

/* Complementarity residual of x in velocity units (0 at an exact solution):
 * free rows |s|, rows at the lower bound max(s, 0), at the upper bound
 * max(-s, 0), plus any bound violation scaled by A_rr; s = b - A x. */
static double lcp_residual(int n, const double* A, int lda, const double* b, const double* lo, const double* hi,
                           const int* findex, double mu, const double* x, double tol_x)
{
    double res = 0.0;
    for (int r = 0; r < n; ++r) {
        double s = b[r];
        for (int c = 0; c < n; ++c) s -= A[r * lda + c] * x[c];
        double l, u, e;
        row_bounds(r, lo, hi, findex, mu, x, &l, &u);
        if (x[r] < l - tol_x || x[r] > u + tol_x)
            e = (x[r] < l ? l - x[r] : x[r] - u) * A[r * lda + r];
        else if (u - l <= tol_x)
            e = 0.0;  /* a pinned row (friction of a contact without normal impulse) */
        else if (x[r] <= l + tol_x)
            e = s > 0.0 ? s : 0.0;
        else if (x[r] >= u - tol_x)
            e = s < 0.0 ? -s : 0.0;
        else
            e = fabs(s);
        res = e > res ? e : res;
    }
    return res;
}

/* Exact solve of the box QP  min 1/2 x'Ax - b'x,  L <= x <= U  (A symmetric
 * positive definite: the CFM makes it so) by the primal active-set method,
 * warm-started from x (clamped).  Finite for a strictly convex QP: every
 * step either reaches the minimiser on the working set (then the bound with
 * the most wrongly signed multiplier is released) or stops at the first
 * blocking bound, which joins the working set.  Returns the iterations
 * used, or -1 when the budget ran out. */
static int boxqp_solve(int n, const double* A, int lda, const double* b, const double* L, const double* U,
                       double* x)
{
    static _Thread_local double K[OR_LCP_MAXN * OR_LCP_MAXN];
    double g[OR_LCP_MAXN], c[OR_LCP_MAXN], d[OR_LCP_MAXN];
    int fidx[OR_LCP_MAXN], ws[OR_LCP_MAXN]; /* ws: 0 free, 1 held at L, 2 held at U */
    for (int r = 0; r < n; ++r) {
        if (x[r] <= L[r]) { x[r] = L[r]; ws[r] = 1; }
        else if (x[r] >= U[r]) { x[r] = U[r]; ws[r] = 2; }
        else ws[r] = 0;
        if (L[r] == U[r]) ws[r] = 1;
    }
    int at_min = 0;  /* the last step was a full Newton step: x minimises the working set */
    for (int it = 0; it < 4 * n + 50; ++it) {
        for (int r = 0; r < n; ++r) {
            double acc = -b[r];
            for (int e = 0; e < n; ++e) acc += A[r * lda + e] * x[e];
            g[r] = acc;
        }
        int nf = 0;
        for (int r = 0; r < n; ++r)
            if (ws[r] == 0) fidx[nf++] = r;
        /* Newton step on the free rows: A_FF d_F = -g_F */
        for (int i = 0; i < nf; ++i) {
            for (int j = 0; j < nf; ++j) K[i * nf + j] = A[fidx[i] * lda + fidx[j]];
            c[i] = -g[fidx[i]];
        }
        double dn = 0.0;
        if (nf > 0 && !at_min) {
            if (!lcp_gauss(nf, K, c, d)) return -1;
            for (int i = 0; i < nf; ++i) dn = fabs(d[i]) > dn ? fabs(d[i]) : dn;
        }
        double xm = 0.0;
        for (int r = 0; r < n; ++r) xm = fabs(x[r]) > xm ? fabs(x[r]) : xm;
        if (at_min || dn <= 1e-15 * (1.0 + xm)) {
            at_min = 0;
            /* minimiser on the working set: release the worst multiplier */
            int worst = -1;
            double wv = 0.0;
            double gm = 0.0;
            for (int r = 0; r < n; ++r) gm = fabs(g[r]) > gm ? fabs(g[r]) : gm;
            const double tol = 1e-13 * (1.0 + gm);
            for (int r = 0; r < n; ++r) {
                if (L[r] == U[r]) continue;
                const double v = (ws[r] == 1) ? -g[r] : ((ws[r] == 2) ? g[r] : 0.0);
                if (v > tol && v > wv) { wv = v; worst = r; }
            }
            if (worst < 0) return it;
            ws[worst] = 0;
            continue;
        }
        /* longest feasible step along d (at most 1) */
        double alpha = 1.0;
        int block = -1, bside = 0;
        for (int i = 0; i < nf; ++i) {
            const int r = fidx[i];
            if (d[i] < 0.0 && x[r] + d[i] < L[r]) {
                const double a = (L[r] - x[r]) / d[i];
                if (a < alpha) { alpha = a; block = r; bside = 1; }
            } else if (d[i] > 0.0 && x[r] + d[i] > U[r]) {
                const double a = (U[r] - x[r]) / d[i];
                if (a < alpha) { alpha = a; block = r; bside = 2; }
            }
        }
        if (alpha < 0.0) alpha = 0.0;
        for (int i = 0; i < nf; ++i) x[fidx[i]] += alpha * d[i];
        if (block >= 0) {
            x[block] = (bside == 1) ? L[block] : U[block];
            ws[block] = bside;
        } else {
            at_min = 1;
        }
    }
    return -1;
}

/* Converged mode: DART's boxed LCP.  BoxedLcpConstraintSolver hands the
 * constraint rows to DantzigBoxedLcpSolver, i.e. ODE's dSolveLCP
 * (dart/external/odelcpsolver/lcp.cpp; the reference installs it as
 * libdart-external-odelcpsolver-dev, .docker/cicd-devel.Dockerfile:56-60)
 * [EXT].  Its friction-index handling fixes the answer: the rows with
 * findex >= 0 are permuted to the end; the pivoting solves the other rows
 * first (normals in [0, inf), joint rows in their boxes, friction impulses
 * still 0), and on reaching the first friction row it sets EVERY friction
 * row's box once to +-|mu x_n| from the normal impulses solved so far
 * (x_n = 0: the row is pinned at 0) and never updates it; the remaining
 * pivots keep every row complementary with those boxes.  A is symmetric
 * positive definite (the CFM), so each stage is a strictly convex box QP
 * with a unique minimiser, whatever the pivoting order:
 *   stage 1: x_S = argmin over the non-friction rows S, friction impulses 0;
 *   stage 2: x = argmin over all rows, friction boxes [-mu x_n1, mu x_n1]
 *            from the stage-1 normals.
 * Both solved exactly here (boxqp_solve, warm-started from x).  The result
 * is not the fixed point of the friction boxes (|x_t| <= mu x_n at the FINAL
 * normals): where the friction saturates and the contact's normals shift
 * with it (a sliding, pitching foot) DART keeps the boxes of the
 * frictionless normals.  Stats: boxqp iterations of both stages; the final
 * complementarity residual of the two stages' boxes (velocity units), < 0
 * when a stage ran out of budget. */
/* Conditioning probe (tests only): with eps > 0 every exact LCP solve sees A
 * with each symmetric pair of entries scaled by (1 + eps u), u uniform in
 * [-1, 1) from a per-call LCG stream -- the perturbation storing A in fp32
 * makes (eps ~ 6e-8).  An LCP whose answer moves as much under it as the
 * GPU's differs from the fp64 one is ill-conditioned at fp32, not solved
 * wrong. */
static _Thread_local double g_lcp_eps = 0.0;
static _Thread_local uint64_t g_lcp_seed = 0;

void or_set_lcp_perturbation(double eps, uint64_t seed)
{
    g_lcp_eps = eps;
    g_lcp_seed = seed;
}

static void lcp_dantzig_exact(int n, const double* A, int lda, const double* b, const double* lo,
                              const double* hi, const int* findex, double mu, double* x);

static void lcp_dantzig(int n, const double* A, int lda, const double* b, const double* lo, const double* hi,
                        const int* findex, double mu, double* x)
{
    if (g_lcp_eps <= 0.0 || n > OR_LCP_MAXN) {
        lcp_dantzig_exact(n, A, lda, b, lo, hi, findex, mu, x);
        return;
    }
    static _Thread_local double Ap[OR_LCP_MAXN * OR_LCP_MAXN];
    uint64_t st = g_lcp_seed * 6364136223846793005ull + 1442695040888963407ull;
    for (int r = 0; r < n; ++r)
        for (int c = r; c < n; ++c) {
            st = st * 6364136223846793005ull + 1442695040888963407ull;
            const double u = (double)(st >> 11) * (2.0 / 9007199254740992.0) - 1.0;
            const double v = A[r * lda + c] * (1.0 + g_lcp_eps * u);
            Ap[r * n + c] = v;
            Ap[c * n + r] = v;
        }
    lcp_dantzig_exact(n, Ap, n, b, lo, hi, findex, mu, x);
}

static void lcp_dantzig_exact(int n, const double* A, int lda, const double* b, const double* lo,
                              const double* hi, const int* findex, double mu, double* x)
{
    static _Thread_local double As[OR_LCP_MAXN * OR_LCP_MAXN];
    double bs[OR_LCP_MAXN], Ls[OR_LCP_MAXN], Us[OR_LCP_MAXN], xs[OR_LCP_MAXN], L[OR_LCP_MAXN] = {0}, U[OR_LCP_MAXN] = {0};
    int sidx[OR_LCP_MAXN], nofric[OR_LCP_MAXN];
    int ns = 0, failed = 0, iters = 0;
    for (int r = 0; r < n; ++r) {
        nofric[r] = -1;
        if (findex[r] < 0) sidx[ns++] = r;
    }
    /* stage 1: the non-friction rows, friction impulses 0 */
    for (int i = 0; i < ns; ++i) {
        const int r = sidx[i];
        for (int j = 0; j < ns; ++j) As[i * ns + j] = A[r * lda + sidx[j]];
        bs[i] = b[r];
        Ls[i] = lo[r];
        Us[i] = hi[r];
        xs[i] = x[r];
    }
    if (ns > 0) {
        const int it = boxqp_solve(ns, As, ns, bs, Ls, Us, xs);
        if (it < 0) failed = 1; else iters += it;
    }
    double x1[OR_LCP_MAXN];
    for (int r = 0; r < n; ++r) x1[r] = 0.0;
    for (int i = 0; i < ns; ++i) x1[sidx[i]] = xs[i];
    for (int r = 0; r < n && r < OR_CAP_MAXN + 64; ++r) g_last_x1[r] = x1[r];
    const double res1 = ns > 0 ? lcp_residual(ns, As, ns, bs, Ls, Us, nofric, 0.0, xs, 1e-12) : 0.0;
    /* stage 2: friction boxes from the stage-1 normals, all rows */
    for (int r = 0; r < n; ++r) {
        if (findex[r] >= 0) {
            const double xn = x1[findex[r]];
            const double u = xn > 0.0 ? fabs(mu * xn) : 0.0;
            L[r] = -u;
            U[r] = u;
        } else {
            L[r] = lo[r];
            U[r] = hi[r];
            x[r] = x1[r];
        }
    }
    const int it2 = boxqp_solve(n, A, lda, b, L, U, x);
    if (it2 < 0) failed = 1; else iters += it2;
    double xm = 0.0;
    for (int r = 0; r < n; ++r) xm = fabs(x[r]) > xm ? fabs(x[r]) : xm;
    const double res2 = lcp_residual(n, A, lda, b, L, U, nofric, 0.0, x, 1e-12 * (1.0 + xm));
    g_pgs_delta = res1 > res2 ? res1 : res2;
    if (failed) g_pgs_delta = -1.0 - g_pgs_delta;
    g_pgs_sweeps += 1000000 * iters;
}

void or_pgs(int n, const double* A, const double* b, const double* lo,
            const double* hi, double* x, int iters)
{
    g_pgs_sweeps = 0;
    for (int it = 0; it < pgs_budget(iters); ++it) {
        for (int r = 0; r < n; ++r) {
            double s = b[r];
            for (int c = 0; c < n; ++c) s -= A[r * n + c] * x[c];
            double v = x[r] + s / A[r * n + r];
            if (v < lo[r]) v = lo[r];
            if (v > hi[r]) v = hi[r];
            x[r] = v;
        }
        pgs_count(it);
    }
    if (iters < 0 && n <= OR_LCP_MAXN) {
        int findex[OR_LCP_MAXN];
        for (int r = 0; r < n; ++r) findex[r] = -1;
        lcp_dantzig(n, A, n, b, lo, hi, findex, 0.0, x);
    }
}

/* DART constants [EXT]: DART_ERP 0.01, DART_MAX_ERV 10, DART_CFM 1e-9,
 * DART_ERROR_ALLOWANCE 0. */
#define OR_ERP 0.01
#define OR_MAX_ERV 10.0
#define OR_CFM 1e-9

int or_step(const or_model* m, double dt, double* q, double* qd,
            const int32_t* mode, const double* cmd, int pgs_iters,
            double* qdd_out, double* force_out)
{
    const int n = m->n;
    double tau[OR_MAXB] = {0}, qdd[OR_MAXB] = {0};
    or_impulse_factor fac;

    /* GenericJoint::setCommand (FORCE): clip to the effort limits */
    for (int i = 0; i < n; ++i) {
        double t = 0.0;
        if (mode[i] == OR_FORCE) {
            t = cmd[i];
            if (t < -m->effort[i]) t = -m->effort[i];
            if (t > m->effort[i]) t = m->effort[i];
        }
        tau[i] = t;
    }

    aba_full(m, q, qd, tau, dt, qdd, &fac);
    for (int i = 0; i < n; ++i) qd[i] += dt * qdd[i];

    /* constraint rows: limit, servo, Coulomb friction (per joint, body order) */
    int rd[3 * OR_MAXB];
    double b[3 * OR_MAXB], lo[3 * OR_MAXB], hi[3 * OR_MAXB];
    int nr = 0;
    for (int i = 0; i < n; ++i) {
        if (m->limited[i]) {
            double viol = q[i] - m->lower[i];
            int active = 0;
            if (viol <= 0.0) { lo[nr] = 0.0; hi[nr] = INFINITY; active = 1; }
            else {
                viol = q[i] - m->upper[i];
                if (viol >= 0.0) { lo[nr] = -INFINITY; hi[nr] = 0.0; active = 1; }
            }
            if (active) {
                double bounce = -viol * OR_ERP / dt;
                if (bounce > OR_MAX_ERV) bounce = OR_MAX_ERV;
                if (bounce < -OR_MAX_ERV) bounce = -OR_MAX_ERV;
                b[nr] = -qd[i] + bounce;
                rd[nr++] = i;
            }
        }
        if (mode[i] == OR_SERVO) {
            double vc = cmd[i];
            if (vc < -m->vel_limit[i]) vc = -m->vel_limit[i];
            if (vc > m->vel_limit[i]) vc = m->vel_limit[i];
            const double err = vc - qd[i];
            if (err != 0.0) {
                b[nr] = err;
                lo[nr] = -m->effort[i] * dt;
                hi[nr] = m->effort[i] * dt;
                rd[nr++] = i;
            }
        }
        if (m->friction[i] != 0.0 && qd[i] != 0.0) {
            b[nr] = -qd[i];
            hi[nr] = m->friction[i] * dt;
            lo[nr] = -hi[nr];
            rd[nr++] = i;
        }
    }

    double imp[OR_MAXB];
    for (int i = 0; i < n; ++i) imp[i] = 0.0;
    if (nr > 0) {
        double cols[OR_MAXB][OR_MAXB];
        int have[OR_MAXB];
        for (int i = 0; i < n; ++i) have[i] = 0;
        for (int r = 0; r < nr; ++r)
            if (!have[rd[r]]) { impulse_column(m, &fac, rd[r], cols[rd[r]]); have[rd[r]] = 1; }
        double A[9 * OR_MAXB * OR_MAXB];
        double x[3 * OR_MAXB];
        for (int r = 0; r < nr; ++r) {
            for (int c = 0; c < nr; ++c) A[r * nr + c] = cols[rd[c]][rd[r]];
            A[r * nr + r] *= (1.0 + OR_CFM);
            x[r] = 0.0;
        }
        or_pgs(nr, A, b, lo, hi, x, pgs_iters);
        for (int r = 0; r < nr; ++r) imp[rd[r]] += x[r];
        double dqd[OR_MAXB];
        for (int i = 0; i < n; ++i) dqd[i] = 0.0;
        for (int i = 0; i < n; ++i)
            if (imp[i] != 0.0)
                for (int k = 0; k < n; ++k) dqd[k] += cols[i][k] * imp[i];
        for (int i = 0; i < n; ++i) {
            qd[i] += dqd[i];
            qdd[i] += dqd[i] / dt;
        }
    }

    integrate_joint_positions(m, q, qd, dt);
    if (qdd_out)
        for (int i = 0; i < n; ++i) qdd_out[i] = qdd[i];
    if (force_out)
        for (int i = 0; i < n; ++i) force_out[i] = tau[i] + imp[i] / dt;
    return nr;
}

/* ---------------- free body + ground contacts ---------------- */

/* DART 6 ContactConstraint defaults [EXT, restated, parity unpinned]:
 * error-reduction parameter 0.01, max error-reduction velocity 1e-3,
 * constraint force mixing 1e-5, error allowance 0, restitution 0; friction
 * is a pyramid over the two ODE plane-space tangents (dPlaneSpace), each
 * bounded by mu times the normal impulse ("findex"). */
#define OR_C_ERP 0.01
#define OR_C_MAX_ERV 1e-3
#define OR_C_CFM 1e-5

/* exp of se(3) (DART math::expMap): R = Rodrigues(phi), t = V(phi) u with
 * V = 1 + (1 - cos th)/th^2 [phi]x + (th - sin th)/th^3 [phi]x^2 */
static void se3_exp(const double phi[3], const double u[3], double R[9], double t[3])
{
    const double th2 = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
    const double th = sqrt(th2);
    double a, b, c; /* R = 1 + a K + b K^2,  V = 1 + b K + c K^2 */
    if (th < 1e-8) {
        a = 1.0 - th2 / 6.0;
        b = 0.5 - th2 / 24.0;
        c = 1.0 / 6.0 - th2 / 120.0;
    } else {
        a = sin(th) / th;
        b = (1.0 - cos(th)) / th2;
        c = (th - sin(th)) / (th2 * th);
    }
    const double K[9] = {0, -phi[2], phi[1], phi[2], 0, -phi[0], -phi[1], phi[0], 0};
    double K2[9];
    for (int r = 0; r < 3; ++r)
        for (int q = 0; q < 3; ++q) {
            double acc = 0.0;
            for (int k = 0; k < 3; ++k) acc += K[r * 3 + k] * K[k * 3 + q];
            K2[r * 3 + q] = acc;
        }
    for (int k = 0; k < 9; ++k) R[k] = (k % 4 == 0 ? 1.0 : 0.0) + a * K[k] + b * K2[k];
    for (int r = 0; r < 3; ++r) {
        double acc = u[r];
        for (int k = 0; k < 3; ++k) acc += (b * K[r * 3 + k] + c * K2[r * 3 + k]) * u[k];
        t[r] = acc;
    }
}

/* ODE dPlaneSpace: two unit vectors spanning the plane orthogonal to n */
static void plane_space(const double n[3], double p[3], double q[3])
{
    if (fabs(n[2]) > 0.7071067811865476) {
        const double a = n[1] * n[1] + n[2] * n[2], k = 1.0 / sqrt(a);
        p[0] = 0; p[1] = -n[2] * k; p[2] = n[1] * k;
        q[0] = a * k; q[1] = -n[0] * p[2]; q[2] = n[0] * p[1];
    } else {
        const double a = n[0] * n[0] + n[1] * n[1], k = 1.0 / sqrt(a);
        p[0] = -n[1] * k; p[1] = n[0] * k; p[2] = 0;
        q[0] = -n[2] * p[1]; q[1] = n[2] * p[0]; q[2] = a * k;
    }
}

/* solve the 6x6 SPD system A x = b (Gaussian elimination, partial pivoting) */
static void solve6(const double* A_in, const double* b, double* x)
{
    double A[36], y[6];
    memcpy(A, A_in, sizeof A);
    memcpy(y, b, sizeof y);
    for (int c = 0; c < 6; ++c) {
        int piv = c;
        for (int r = c + 1; r < 6; ++r)
            if (fabs(A[r * 6 + c]) > fabs(A[piv * 6 + c])) piv = r;
        if (piv != c) {
            for (int k = 0; k < 6; ++k) { double t = A[c * 6 + k]; A[c * 6 + k] = A[piv * 6 + k]; A[piv * 6 + k] = t; }
            double t = y[c]; y[c] = y[piv]; y[piv] = t;
        }
        for (int r = c + 1; r < 6; ++r) {
            const double f = A[r * 6 + c] / A[c * 6 + c];
            for (int k = c; k < 6; ++k) A[r * 6 + k] -= f * A[c * 6 + k];
            y[r] -= f * y[c];
        }
    }
    for (int r = 5; r >= 0; --r) {
        double acc = y[r];
        for (int k = r + 1; k < 6; ++k) acc -= A[r * 6 + k] * x[k];
        x[r] = acc / A[r * 6 + r];
    }
}

int or_free_step(const or_free_model* m, double dt, or_free_state* s, int pgs_iters,
                 double* c_pos, double* c_normal, double* c_force, double* c_depth)
{
    /* spatial inertia about the body origin, [angular; linear] */
    double I[36];
    {
        const double ms = m->mass, *c = m->com, *ic = m->Ic;
        const double Icm[9] = {ic[0], ic[3], ic[4], ic[3], ic[1], ic[5], ic[4], ic[5], ic[2]};
        const double C[9] = {0, -c[2], c[1], c[2], 0, -c[0], -c[1], c[0], 0};
        m6_zero(I);
        for (int r = 0; r < 3; ++r)
            for (int k = 0; k < 3; ++k) {
                double cc = 0.0;
                for (int j = 0; j < 3; ++j) cc -= C[r * 3 + j] * C[j * 3 + k];
                I[r * 6 + k] = Icm[r * 3 + k] + ms * cc;
                I[r * 6 + k + 3] = ms * C[r * 3 + k];
                I[(r + 3) * 6 + k] = -ms * C[r * 3 + k];
                I[(r + 3) * 6 + k + 3] = (r == k) ? ms : 0.0;
            }
    }
    const double* R = s->R;
    double V[6] = {s->w[0], s->w[1], s->w[2], s->v[0], s->v[1], s->v[2]};
    /* forward dynamics (FreeJoint = ABA on one body): I a = dad(V, I V) + I [0; g_b] */
    double gb[3], IV[6], dd[6], ga[6] = {0}, Ig[6], f[6], a[6];
    for (int r = 0; r < 3; ++r) gb[r] = R[r] * m->gravity[0] + R[3 + r] * m->gravity[1] + R[6 + r] * m->gravity[2];
    m6_vec(I, V, IV);
    sp_dad(V, IV, dd);
    ga[3] = gb[0]; ga[4] = gb[1]; ga[5] = gb[2];
    m6_vec(I, ga, Ig);
    for (int k = 0; k < 6; ++k) f[k] = dd[k] + Ig[k];
    solve6(I, f, a);
    for (int k = 0; k < 6; ++k) V[k] += dt * a[k];

    /* collision detection against the ground plane z = 0 (positions of the
     * start of the step, velocities after integrateVelocities) */
    int nc = 0;
    double cb[OR_MAXCONTACTS][3], depth[OR_MAXCONTACTS], cw[OR_MAXCONTACTS][3];
    if (m->ground) {
        for (int k = 0; k < m->n_shapes; ++k) {
            const double* h = m->shape_size[k];
            const double* SR = m->shape_R[k];
            const double* sp = m->shape_p[k];
            if (m->shape_type[k] != 1) {
                double RS[9];
                rot_mul(R, SR, RS);
                const int corners = (m->shape_type[k] == 3) ? m->mesh_npts[k] : 8;
                for (int corner = 0; corner < corners; ++corner) {
                    double l[3];
                    if (m->shape_type[k] == 3)   /* mesh entry: its support points */
                        memcpy(l, m->mesh_pt[k][corner], sizeof l);
                    else
                        or_slot_point(m->shape_type[k], h, RS, corner, l);
                    double b[3], x[3];
                    for (int r = 0; r < 3; ++r) b[r] = sp[r] + SR[r * 3] * l[0] + SR[r * 3 + 1] * l[1] + SR[r * 3 + 2] * l[2];
                    for (int r = 0; r < 3; ++r) x[r] = s->p[r] + R[r * 3] * b[0] + R[r * 3 + 1] * b[1] + R[r * 3 + 2] * b[2];
                    if (x[2] < 0.0) {
                        memcpy(cb[nc], b, sizeof b);
                        memcpy(cw[nc], x, sizeof x);
                        depth[nc] = -x[2];
                        ++nc;
                    }
                }
            } else {
                double x[3];
                for (int r = 0; r < 3; ++r) x[r] = s->p[r] + R[r * 3] * sp[0] + R[r * 3 + 1] * sp[1] + R[r * 3 + 2] * sp[2];
                if (x[2] - h[0] < 0.0) {
                    /* lowest point of the sphere */
                    double xw[3] = {x[0], x[1], x[2] - h[0]}, d[3], bb[3];
                    for (int r = 0; r < 3; ++r) d[r] = xw[r] - s->p[r];
                    for (int r = 0; r < 3; ++r) bb[r] = R[r] * d[0] + R[3 + r] * d[1] + R[6 + r] * d[2];
                    memcpy(cb[nc], bb, sizeof bb);
                    memcpy(cw[nc], xw, sizeof xw);
                    depth[nc] = h[0] - x[2];
                    ++nc;
                }
            }
        }
    }

    double x[3 * OR_MAXCONTACTS];
    const double n[3] = {0, 0, 1};
    double t1[3], t2[3];
    plane_space(n, t1, t2);
    if (nc > 0) {
        /* rows: (normal, t1, t2) per contact; J = [c x d_b; d_b] in the body frame */
        const int nr = 3 * nc;
        double J[3 * OR_MAXCONTACTS][6], MJ[3 * OR_MAXCONTACTS][6], b[3 * OR_MAXCONTACTS];
        for (int i = 0; i < nc; ++i)
            for (int d = 0; d < 3; ++d) {
                const double* dw = (d == 0) ? n : (d == 1 ? t1 : t2);
                double db[3];
                for (int r = 0; r < 3; ++r) db[r] = R[r] * dw[0] + R[3 + r] * dw[1] + R[6 + r] * dw[2];
                double* Jr = J[3 * i + d];
                cross3(cb[i], db, Jr);
                Jr[3] = db[0]; Jr[4] = db[1]; Jr[5] = db[2];
                solve6(I, Jr, MJ[3 * i + d]);
                const double vrel = dot6(Jr, V);
                double bounce = 0.0;
                if (d == 0) {
                    bounce = OR_C_ERP * depth[i] / dt;
                    if (bounce > OR_C_MAX_ERV) bounce = OR_C_MAX_ERV;
                }
                b[3 * i + d] = -vrel + bounce;
            }
        double A[3 * OR_MAXCONTACTS][3 * OR_MAXCONTACTS];
        for (int r = 0; r < nr; ++r)
            for (int c = 0; c < nr; ++c) A[r][c] = dot6(J[r], MJ[c]);
        for (int r = 0; r < nr; ++r) { A[r][r] *= (1.0 + OR_C_CFM); x[r] = 0.0; }
        g_pgs_sweeps = 0;
        for (int it = 0; it < pgs_budget(pgs_iters); ++it) {
            for (int r = 0; r < nr; ++r) {
                double acc = b[r];
                for (int c = 0; c < nr; ++c) acc -= A[r][c] * x[c];
                double v = x[r] + acc / A[r][r];
                double lo, hi;
                if (r % 3 == 0) { lo = 0.0; hi = INFINITY; }
                else { hi = m->mu * x[r - r % 3]; lo = -hi; }
                if (v < lo) v = lo;
                if (v > hi) v = hi;
                x[r] = v;
            }
            pgs_count(it);
        }
        if (pgs_iters < 0) {
            double lo[3 * OR_MAXCONTACTS], hi[3 * OR_MAXCONTACTS];
            int findex[3 * OR_MAXCONTACTS];
            for (int r = 0; r < nr; ++r) {
                lo[r] = 0.0;
                hi[r] = INFINITY;
                findex[r] = (r % 3 == 0) ? -1 : r - r % 3;
            }
            lcp_dantzig(nr, &A[0][0], 3 * OR_MAXCONTACTS, b, lo, hi, findex, m->mu, x);
        }
        for (int r = 0; r < nr; ++r)
            for (int k = 0; k < 6; ++k) V[k] += MJ[r][k] * x[r];
    }

    /* integratePositions: T <- T exp(dt V) */
    double phi[3] = {dt * V[0], dt * V[1], dt * V[2]}, u[3] = {dt * V[3], dt * V[4], dt * V[5]};
    double dR[9], dp[3], Rn[9];
    se3_exp(phi, u, dR, dp);
    for (int r = 0; r < 3; ++r) {
        s->p[r] += R[r * 3] * dp[0] + R[r * 3 + 1] * dp[1] + R[r * 3 + 2] * dp[2];
        for (int q = 0; q < 3; ++q)
            Rn[r * 3 + q] = R[r * 3] * dR[q] + R[r * 3 + 1] * dR[3 + q] + R[r * 3 + 2] * dR[6 + q];
    }
    memcpy(s->R, Rn, sizeof Rn);
    for (int k = 0; k < 3; ++k) { s->w[k] = V[k]; s->v[k] = V[3 + k]; }

    for (int i = 0; i < nc; ++i) {
        for (int r = 0; r < 3; ++r) {
            if (c_pos) c_pos[3 * i + r] = cw[i][r];
            if (c_normal) c_normal[3 * i + r] = n[r];
            if (c_force) c_force[3 * i + r] = (n[r] * x[3 * i] + t1[r] * x[3 * i + 1] + t2[r] * x[3 * i + 2]) / dt;
        }
        if (c_depth) c_depth[i] = depth[i];
    }
    return nc;
}

/* ---------------- joint PID (ign-math 6 PID, [EXT]) ---------------- */

/* ignition::math::PID::Update restated [EXT: ign-math6 src/PID.cc, not
 * vendored]: error = current - reference (JointController.cpp), the
 * integral is clamped to [iMin, iMax] and the command to [cmdMin, cmdMax]
 * when those ranges are non-empty; a zero dt returns 0 and leaves the state
 * unchanged.  Reset() zeroes pErrLast / iErr / cmd. */
double or_pid_update(const or_pid_gains* g, or_pid_state* s, double err, double dt)
{
    if (dt == 0.0 || isnan(err) || isinf(err)) return 0.0;
    const double pterm = g->p * err;
    s->ierr = s->ierr + g->i * dt * err;
    if (g->imax >= g->imin) {
        if (s->ierr > g->imax) s->ierr = g->imax;
        if (s->ierr < g->imin) s->ierr = g->imin;
    }
    const double derr = (err - s->perr_last) / dt;
    s->perr_last = err;
    double cmd = -pterm - s->ierr - g->d * derr + g->offset;
    if (g->cmdmax >= g->cmdmin) {
        if (cmd > g->cmdmax) cmd = g->cmdmax;
        if (cmd < g->cmdmin) cmd = g->cmdmin;
    }
    s->cmd = cmd;
    return cmd;
}

/* ---------------- Philox4x32-10 ---------------- */

void or_philox(uint64_t seed, uint32_t world, uint32_t episode, uint32_t out[4])
{
    const uint32_t ctr[4] = {world, episode, 0u, 0u};
    const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    or_philox_raw(ctr, key, out);
}

void or_philox_raw(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4])
{
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static double u01(uint32_t x) { return (double)(x >> 8) * (1.0 / 16777216.0); }
static double unif(uint32_t x, double lo, double hi) { return lo + (hi - lo) * u01(x); }

/* float32 bounds as gym.spaces.Box(dtype=float32) stores them */
static double f32(double v) { return (double)(float)v; }

#define OR_PI 3.14159265358979323846
static double deg2rad(double d) { return d * OR_PI / 180.0; }

/* Philox4x32-10 with the third counter word set (block index) */
static void philox_block(uint64_t seed, uint32_t world, uint32_t episode, uint32_t block, uint32_t out[4])
{
    const uint32_t ctr[4] = {world, episode, block, 0u};
    const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    or_philox_raw(ctr, key, out);
}

/* SDFRandomizer.sample (randomizers/model/sdf.py:264-315): an Additive
 * Uniform randomisation with force_positive clips the SAMPLE at 0, so every
 * moving body's mass becomes m + max(U(low, high), 0) (cartpole.py:100-135;
 * Philox blocks 1.., four bodies per block); the physics randomizer sets the
 * gravity to (0, 0, N(mean, std)) (cartpole.py:51-56; Box-Muller on block 8). */
void or_task_sample_physics(const or_model* m, const or_task* t, uint32_t world,
                            uint32_t episode, double* masses, double* gz)
{
    for (int i = 0; i < m->n; ++i) masses[i] = m->mass[i];
    *gz = 0.0;
    if (t->randomize & 1) {
        for (int b = 0; b < (m->n + 3) / 4; ++b) {
            uint32_t r[4];
            philox_block(t->seed, world, episode, 1u + (uint32_t)b, r);
            for (int k = 0; k < 4 && 4 * b + k < m->n; ++k) {
                double u = t->mass_low + (t->mass_high - t->mass_low) * ((double)(r[k] >> 8) * (1.0 / 16777216.0));
                masses[4 * b + k] += (u > 0.0) ? u : 0.0;
            }
        }
    }
    if (t->randomize & 2) {
        uint32_t r[4];
        philox_block(t->seed, world, episode, 8u, r);
        const double u1 = (double)((r[0] >> 8) + 1u) * (1.0 / 16777216.0);
        const double u2 = (double)(r[1] >> 8) * (1.0 / 16777216.0);
        *gz = t->gravity_mean + t->gravity_std * sqrt(-2.0 * log(u1)) * cos(2.0 * 3.14159265358979323846 * u2);
    }
}

/* the model one world steps with: the shared one, or a copy carrying the
 * world's randomised masses / gravity */
static const or_model* world_model(const or_model* m, const or_task* t, uint32_t w, uint32_t ep,
                                   or_model* scratch)
{
    if (!t->randomize) return m;
    double masses[OR_MAXB], gz;
    or_task_sample_physics(m, t, w, ep, masses, &gz);
    memcpy(scratch, m, sizeof(or_model));
    for (int i = 0; i < m->n; ++i) scratch->mass[i] = masses[i];
    if (t->randomize & 2)
        for (int k = 0; k < 3; ++k) scratch->gravity_base[k] = gz * t->gdir[k];
    return scratch;
}

void or_task_reset_state(const or_task* t, uint32_t world, uint32_t episode,
                         double* q, double* qd)
{
    uint32_t r[4];
    or_philox(t->seed, world, episode, r);
    switch (t->kind) {
    case OR_TASK_CARTPOLE_DISCRETE:
    case OR_TASK_CARTPOLE_CONTINUOUS_BALANCING:
        /* x, dx, q, dq = uniform(-0.05, 0.05, 4)  cartpole_discrete_balancing.py:137 */
        q[0] = unif(r[0], -0.05, 0.05); qd[0] = unif(r[1], -0.05, 0.05);
        q[1] = unif(r[2], -0.05, 0.05); qd[1] = unif(r[3], -0.05, 0.05);
        break;
    case OR_TASK_CARTPOLE_CONTINUOUS_SWINGUP:
        /* q = pi - deg2rad(U(-60, 60)); x, dx, dq = U(-0.05, 0.05)
         * cartpole_continuous_swingup.py:145-146 */
        q[1] = OR_PI - deg2rad(unif(r[0], -60.0, 60.0));
        q[0] = unif(r[1], -0.05, 0.05); qd[0] = unif(r[2], -0.05, 0.05);
        qd[1] = unif(r[3], -0.05, 0.05);
        break;
    case OR_TASK_PENDULUM_SWINGUP: {
        /* cos, sin, dq = observation_space.sample(); q = atan2(sin, cos)
         * pendulum_swingup.py:117-127 */
        const double c = unif(r[0], -1.0, 1.0), s = unif(r[1], -1.0, 1.0);
        q[0] = atan2(s, c);
        qd[0] = unif(r[2], -10.0, 10.0);
        break;
    }
    }
}

int or_task_obs(const or_task* t, const double* q, const double* qd, double* obs)
{
    if (t->kind == OR_TASK_PENDULUM_SWINGUP) {
        obs[0] = cos(q[0]); obs[1] = sin(q[0]); obs[2] = qd[0];
        return 3;
    }
    /* [x, dx, q, dq]  cartpole_discrete_balancing.py:79-92 */
    obs[0] = q[0]; obs[1] = qd[0]; obs[2] = q[1]; obs[3] = qd[1];
    return 4;
}

static int task_done(const or_task* t, const double* obs)
{
    if (t->kind == OR_TASK_PENDULUM_SWINGUP) {
        /* not observation_space.contains(obs), high = [1, 1, 10] */
        return !(fabs(obs[0]) <= 1.0 && fabs(obs[1]) <= 1.0 && fabs(obs[2]) <= f32(10.0));
    }
    const double qth = (t->kind == OR_TASK_CARTPOLE_CONTINUOUS_SWINGUP) ? deg2rad(5 * 360) : deg2rad(12);
    const double hi[4] = {f32(2.4), f32(20.0), f32(qth), f32(deg2rad(3 * 360))};
    for (int k = 0; k < 4; ++k)
        if (!(obs[k] >= -hi[k] && obs[k] <= hi[k])) return 1;
    return 0;
}

static double task_reward(const or_task* t, const double* q, const double* qd,
                          const double* obs, int done)
{
    switch (t->kind) {
    case OR_TASK_CARTPOLE_DISCRETE:
    case OR_TASK_CARTPOLE_CONTINUOUS_BALANCING: {
        /* cartpole_discrete_balancing.py:94-109 (0.9 * x_thr) and
         * cartpole_continuous_balancing.py:107 (1.0 * x_thr) */
        double r = done ? 0.0 : 1.0;
        if (t->reward_cart_at_center) {
            const double f = (t->kind == OR_TASK_CARTPOLE_DISCRETE) ? 0.9 : 1.0;
            r = r - 0.10 * fabs(obs[0]) - 0.10 * fabs(obs[1]) - 10.0 * (obs[0] >= f * 2.4 ? 1.0 : 0.0);
        }
        return r;
    }
    case OR_TASK_CARTPOLE_CONTINUOUS_SWINGUP: {
        /* cartpole_continuous_swingup.py:116-127 */
        double r = (cos(q[1]) + 1.0) / 2.0;
        r -= 0.1 * qd[0] * qd[0];
        r -= 10.0 * (q[0] >= 0.8 * 2.4 ? 1.0 : 0.0);
        return r;
    }
    case OR_TASK_PENDULUM_SWINGUP: {
        /* pendulum_swingup.py:73-90.  The force target it reads is the
         * JointForceCmd that UpdateSim zero-filled after the run
         * (Physics.cpp:2250-2254), so the tau^2 term is identically 0. */
        double cost = done ? 100.0 : 0.0;
        const double tau_after_run = 0.0;
        cost += q[0] * q[0] + 0.1 * qd[0] * qd[0] + 0.001 * tau_after_run * tau_after_run;
        return -cost;
    }
    }
    return 0.0;
}

static void world_step(const or_model* m, const or_task* t, double* q, double* qd,
                       double action, int pgs_iters)
{
    int32_t mode[OR_MAXB];
    double cmd[OR_MAXB];
    const int drive = 0; /* CartPole "linear" and Pendulum "pivot" are dof 0 */
    for (int i = 0; i < m->n; ++i) { mode[i] = OR_PASSIVE; cmd[i] = 0.0; }
    /* the driven joint ("linear" / "pivot") is in Force mode; the CartPole
     * pivot stays Idle (passive) -- cartpole_discrete_balancing.py:121-131 */
    mode[drive] = OR_FORCE;
    for (int s = 0; s < t->steps_per_run; ++s) {
        /* a force command acts on the first substep only: UpdateSim zero-fills
         * JointForceCmd after every Update (Physics.cpp:2250-2254) */
        cmd[drive] = (s == 0) ? action : 0.0;
        or_step(m, t->dt, q, qd, mode, cmd, pgs_iters, 0, 0);
    }
}

static void vec_step_one(const or_model* m, const or_task* t, int W, int w,
                         double* q, double* qd, double action, uint32_t* episode,
                         uint32_t* steps, double* obs, double* reward,
                         uint8_t* done, double* terminal_obs, int pgs_iters)
{
    const int n = m->n;
    double qw[OR_MAXB], qdw[OR_MAXB], o[4];
    for (int d = 0; d < n; ++d) { qw[d] = q[d * W + w]; qdw[d] = qd[d * W + w]; }
    or_model scratch;
    world_step(world_model(m, t, (uint32_t)(w + t->world0), episode[w], &scratch), t, qw, qdw, action, pgs_iters);
    const int no = or_task_obs(t, qw, qdw, o);
    const int tdone = task_done(t, o);
    reward[w] = task_reward(t, qw, qdw, o, tdone);
    steps[w] += 1;
    int d_ = tdone;
    if (t->max_episode_steps > 0 && steps[w] >= (uint32_t)t->max_episode_steps) d_ = 1;
    done[w] = (uint8_t)d_;
    if (d_) {
        for (int k = 0; k < no; ++k) terminal_obs[w * no + k] = o[k];
        episode[w] += 1;
        steps[w] = 0;
        or_task_reset_state(t, (uint32_t)(w + t->world0), episode[w], qw, qdw);
        or_task_obs(t, qw, qdw, o);
    }
    for (int k = 0; k < no; ++k) obs[w * no + k] = o[k];
    for (int d = 0; d < n; ++d) { q[d * W + w] = qw[d]; qd[d * W + w] = qdw[d]; }
}

static double action_of(const or_task* t, const void* actions, int idx)
{
    if (t->kind == OR_TASK_CARTPOLE_DISCRETE) {
        const int a = ((const int32_t*)actions)[idx];
        return (a == 1) ? 20.0 : -20.0;   /* _force_mag = 20  cartpole_discrete_balancing.py:32,70 */
    }
    return ((const double*)actions)[idx];
}

void or_vec_step(const or_model* m, const or_task* t, int W, double* q,
                 double* qd, const void* actions, uint32_t* episode,
                 uint32_t* steps, double* obs, double* reward, uint8_t* done,
                 double* terminal_obs, int pgs_iters)
{
    for (int w = 0; w < W; ++w)
        vec_step_one(m, t, W, w, q, qd, action_of(t, actions, w), episode, steps,
                     obs, reward, done, terminal_obs, pgs_iters);
}

void or_vec_reset(const or_model* m, const or_task* t, int W, double* q,
                  double* qd, uint32_t* episode, uint32_t* steps, double* obs)
{
    const int n = m->n;
    for (int w = 0; w < W; ++w) {
        double qw[OR_MAXB], qdw[OR_MAXB], o[4];
        episode[w] = 0;
        steps[w] = 0;
        or_task_reset_state(t, (uint32_t)(w + t->world0), 0u, qw, qdw);
        const int no = or_task_obs(t, qw, qdw, o);
        for (int k = 0; k < no; ++k) obs[w * no + k] = o[k];
        for (int d = 0; d < n; ++d) { q[d * W + w] = qw[d]; qd[d * W + w] = qdw[d]; }
    }
}

void or_vec_rollout(const or_model* m, const or_task* t, int W, int T, double* q,
                    double* qd, const void* actions, uint32_t* episode,
                    uint32_t* steps, double* obs, double* reward, uint8_t* done,
                    double* terminal_obs, int pgs_iters)
{
    for (int s = 0; s < T; ++s) {
        const void* a = (t->kind == OR_TASK_CARTPOLE_DISCRETE)
                            ? (const void*)((const int32_t*)actions + (size_t)s * W)
                            : (const void*)((const double*)actions + (size_t)s * W);
        or_vec_step(m, t, W, q, qd, a, episode, steps, obs, reward, done, terminal_obs,
                    pgs_iters);
    }
}

/* ---------------- articulated floating base + ground contacts ---------------- */

/* Generalized velocity nu = [V0 (base twist, base frame, [w; v]); qd], the
 * coordinates of a DART skeleton whose root joint is a FreeJoint [EXT: DART
 * 6 FreeJoint, relative-twist parameterisation].  Restated densely:
 *   M(q) nu' + h(q, nu) = [0; tau]      (CRBA for M, RNEA for h; Featherstone
 *                                        2008 ch. 6 / 5 with a floating root)
 * DART's implicit joint damping solves (M + dt D) nu' = tau - h - D qd (the
 * recursive ABA of DART applies the same dt*d term to each joint's
 * articulated inertia); constraint impulses use the non-implicit M, as DART's
 * impulse propagation does.  The device kernel runs the recursive form
 * (float_tree.hpp); this dense path is deliberately independent. */

typedef struct {
    double X[OR_MAXB][36];        /* parent -> body (Plucker)             */
    double S[OR_MAXB][6];
    double Rw[OR_MAXB][9], pw[OR_MAXB][3];  /* body pose in the world     */
} or_fkin;

static void float_kin(const or_float_model* m, const or_float_state* s, or_fkin* k)
{
    const or_model* t = &m->tree;
    for (int i = 0; i < t->n; ++i) {
        double R[9], p[3];
        joint_pose(t, i, s->q, R, p);
        plucker(R, p, k->X[i]);
        motion_subspace(t, i, k->S[i]);
        const int pa = t->parent[i];
        const double* Rp = pa < 0 ? s->R : k->Rw[pa];
        const double* pp = pa < 0 ? s->p : k->pw[pa];
        for (int r = 0; r < 3; ++r) {
            k->pw[i][r] = pp[r] + Rp[r * 3] * p[0] + Rp[r * 3 + 1] * p[1] + Rp[r * 3 + 2] * p[2];
            for (int c = 0; c < 3; ++c)
                k->Rw[i][r * 3 + c] = Rp[r * 3] * R[c] + Rp[r * 3 + 1] * R[3 + c] + Rp[r * 3 + 2] * R[6 + c];
        }
    }
}

static void base_inertia(const or_float_model* m, double I[36])
{
    or_model one;
    memset(&one, 0, sizeof one);
    one.n = 1;
    one.mass[0] = m->base_mass;
    memcpy(one.com[0], m->base_com, sizeof m->base_com);
    memcpy(one.Ic[0], m->base_Ic, sizeof m->base_Ic);
    body_inertia(&one, 0, I);
}

void or_float_dynamics(const or_float_model* m, const or_float_state* s, double* M, double* h)
{
    const or_model* t = &m->tree;
    const int n = t->n, nv = 6 + n;
    or_fkin k;
    float_kin(m, s, &k);
    g_cap_n = 0;  /* a step without rows leaves no capture behind */

    /* CRBA: composite inertias accumulate towards the base */
    double Ic[OR_MAXB][36], I0[36];
    for (int i = 0; i < n; ++i) body_inertia(t, i, Ic[i]);
    base_inertia(m, I0);
    for (int i = n - 1; i >= 0; --i) {
        double c[36];
        m6_congruence(k.X[i], Ic[i], c);
        double* dst = t->parent[i] < 0 ? I0 : Ic[t->parent[i]];
        for (int e = 0; e < 36; ++e) dst[e] += c[e];
    }
    for (int e = 0; e < nv * nv; ++e) M[e] = 0.0;
    for (int r = 0; r < 6; ++r)
        for (int c = 0; c < 6; ++c) M[r * nv + c] = I0[r * 6 + c];
    for (int i = 0; i < n; ++i) {
        double F[6];
        m6_vec(Ic[i], k.S[i], F);
        M[(6 + i) * nv + 6 + i] = dot6(k.S[i], F);
        int j = i;
        for (;;) {
            double Fp[6];
            m6t_vec(k.X[j], F, Fp);
            memcpy(F, Fp, sizeof F);
            j = t->parent[j];
            if (j < 0) break;
            M[(6 + i) * nv + 6 + j] = M[(6 + j) * nv + 6 + i] = dot6(k.S[j], F);
        }
        for (int r = 0; r < 6; ++r) M[(6 + i) * nv + r] = M[r * nv + 6 + i] = F[r];
    }

    /* RNEA with nu' = 0; gravity as the base "acceleration" -g0 */
    double g0[3];
    for (int r = 0; r < 3; ++r)
        g0[r] = s->R[r] * m->gravity[0] + s->R[3 + r] * m->gravity[1] + s->R[6 + r] * m->gravity[2];
    const double a0[6] = {0, 0, 0, -g0[0], -g0[1], -g0[2]};
    double V[OR_MAXB][6], a[OR_MAXB][6], f[OR_MAXB][6], f0[6];
    {
        double dd[6], Ib[36], Ia[6], IbV[6];  /* the base's own inertia (I0 is composite) */
        base_inertia(m, Ib);
        m6_vec(Ib, a0, Ia);
        m6_vec(Ib, s->V, IbV);
        sp_dad(s->V, IbV, dd);
        for (int e = 0; e < 6; ++e) f0[e] = Ia[e] - dd[e];
    }
    for (int i = 0; i < n; ++i) {
        const int pa = t->parent[i];
        double Vp[6], ap[6], Sq[6], c[6], I[36], Ia[6], IV[6], dd[6];
        m6_vec(k.X[i], pa < 0 ? s->V : V[pa], Vp);
        m6_vec(k.X[i], pa < 0 ? a0 : a[pa], ap);
        for (int e = 0; e < 6; ++e) { Sq[e] = k.S[i][e] * s->qd[i]; V[i][e] = Vp[e] + Sq[e]; }
        joint_bias(t, i, s->qd, V[i], Sq, c);
        for (int e = 0; e < 6; ++e) a[i][e] = ap[e] + c[e];
        body_inertia(t, i, I);
        m6_vec(I, a[i], Ia);
        m6_vec(I, V[i], IV);
        sp_dad(V[i], IV, dd);
        for (int e = 0; e < 6; ++e) f[i][e] = Ia[e] - dd[e];
    }
    for (int i = n - 1; i >= 0; --i) {
        h[6 + i] = dot6(k.S[i], f[i]);
        double fp[6];
        m6t_vec(k.X[i], f[i], fp);
        double* dst = t->parent[i] < 0 ? f0 : f[t->parent[i]];
        for (int e = 0; e < 6; ++e) dst[e] += fp[e];
    }
    for (int e = 0; e < 6; ++e) h[e] = f0[e];
}

/* dense solve A x = b (n <= 6 + OR_MAXB), partial pivoting */
static void solve_dense(int n, const double* A_in, const double* b, double* x)
{
    double A[(6 + OR_MAXB) * (6 + OR_MAXB)], y[6 + OR_MAXB];
    memcpy(A, A_in, (size_t)n * n * sizeof(double));
    memcpy(y, b, (size_t)n * sizeof(double));
    for (int c = 0; c < n; ++c) {
        int piv = c;
        for (int r = c + 1; r < n; ++r)
            if (fabs(A[r * n + c]) > fabs(A[piv * n + c])) piv = r;
        if (piv != c) {
            for (int e = 0; e < n; ++e) { double tt = A[c * n + e]; A[c * n + e] = A[piv * n + e]; A[piv * n + e] = tt; }
            double tt = y[c]; y[c] = y[piv]; y[piv] = tt;
        }
        for (int r = c + 1; r < n; ++r) {
            const double fr = A[r * n + c] / A[c * n + c];
            for (int e = c; e < n; ++e) A[r * n + e] -= fr * A[c * n + e];
            y[r] -= fr * y[c];
        }
    }
    for (int r = n - 1; r >= 0; --r) {
        double acc = y[r];
        for (int e = r + 1; e < n; ++e) acc -= A[r * n + e] * x[e];
        x[r] = acc / A[r * n + r];
    }
}

/* generalized row of a spatial "direction" f (body-k frame, force-like):
 * J . nu = f . V_k.  f climbs to the base through X^T. */
static void float_row(const or_float_model* m, const or_fkin* k, int body, const double f_in[6], double* J)
{
    const or_model* t = &m->tree;
    const int nv = 6 + t->n;
    double f[6];
    memcpy(f, f_in, sizeof f);
    for (int e = 0; e < nv; ++e) J[e] = 0.0;
    for (int i = body; i >= 0; i = t->parent[i]) {
        J[6 + i] = dot6(k->S[i], f);
        double fp[6];
        m6t_vec(k->X[i], f, fp);
        memcpy(f, fp, sizeof f);
    }
    for (int e = 0; e < 6; ++e) J[e] = f[e];
}

int or_float_step(const or_float_model* m, double dt, or_float_state* s, const int32_t* mode,
                  const double* cmd, int pgs_iters, double* c_pos, double* c_force, double* c_depth,
                  int32_t* c_body)
{
    return or_float_step_warm(m, dt, s, mode, cmd, pgs_iters, 0.0, 0, c_pos, c_force, c_depth, c_body);
}

/* The impulses of the previous step's rows, by row identity: contact slot
 * rows 3 slot + d (d: normal, t1, t2), joint rows OR_WARM_JOINT0 + 3 dof + t
 * (t: limit, servo, Coulomb) -- the kernels' warm-start layout. */
int or_float_step_warm(const or_float_model* m, double dt, or_float_state* s, const int32_t* mode,
                       const double* cmd, int pgs_iters, double pgs_tol, double* warm, double* c_pos,
                       double* c_force, double* c_depth, int32_t* c_body)
{
    const or_model* t = &m->tree;
    const int n = t->n, nv = 6 + n;
    or_fkin k;
    float_kin(m, s, &k);
    g_cap_n = 0;  /* a step without rows leaves no capture behind */

    static _Thread_local double M[(6 + OR_MAXB) * (6 + OR_MAXB)];
    double h[6 + OR_MAXB], rhs[6 + OR_MAXB], acc[6 + OR_MAXB], nu[6 + OR_MAXB];
    or_float_dynamics(m, s, M, h);
    double Mi[(6 + OR_MAXB) * (6 + OR_MAXB)];
    memcpy(Mi, M, (size_t)nv * nv * sizeof(double));
    for (int e = 0; e < 6; ++e) { rhs[e] = -h[e]; nu[e] = s->V[e]; }
    for (int i = 0; i < n; ++i) {
        double tau = 0.0;
        if (mode[i] == OR_FORCE) {
            tau = cmd[i];
            if (tau < -t->effort[i]) tau = -t->effort[i];
            if (tau > t->effort[i]) tau = t->effort[i];
        }
        rhs[6 + i] = tau - h[6 + i] - t->damping[i] * s->qd[i];
        Mi[(6 + i) * nv + 6 + i] += dt * t->damping[i];
        nu[6 + i] = s->qd[i];
    }
    solve_dense(nv, Mi, rhs, acc);
    for (int e = 0; e < nv; ++e) nu[e] += dt * acc[e];

    /* ground contacts (positions of the start of the step), then joint rows
     * -- the order of DART ConstraintSolver::updateConstraints [EXT] */
    int nc = 0;
    double cw[OR_MAXFC][3], depth[OR_MAXFC], cb[OR_MAXFC][3];
    int cbody[OR_MAXFC];
    int slot_id = 0, cslot[OR_MAXFC];
    if (m->ground) {
        for (int sh = 0; sh < m->n_shapes; ++sh) {
            const int bi = m->shape_body[sh];
            const double* Rb = bi < 0 ? s->R : k.Rw[bi];
            const double* pb = bi < 0 ? s->p : k.pw[bi];
            const double* hh = m->shape_size[sh];
            const double* SR = m->shape_R[sh];
            const double* sp = m->shape_p[sh];
            const int corners = (m->shape_type[sh] == 1) ? 1 : 8;
            double RS[9];
            rot_mul(Rb, SR, RS);
            for (int corner = 0; corner < corners; ++corner, ++slot_id) {
                double l[3];
                or_slot_point(m->shape_type[sh], hh, RS, corner, l);
                double b[3], x[3];
                for (int r = 0; r < 3; ++r) b[r] = sp[r] + SR[r * 3] * l[0] + SR[r * 3 + 1] * l[1] + SR[r * 3 + 2] * l[2];
                for (int r = 0; r < 3; ++r) x[r] = pb[r] + Rb[r * 3] * b[0] + Rb[r * 3 + 1] * b[1] + Rb[r * 3 + 2] * b[2];
                double dep = -x[2];
                if (m->shape_type[sh] == 1) {
                    dep = hh[0] - x[2];
                    x[2] -= hh[0];
                    double d[3] = {x[0] - pb[0], x[1] - pb[1], x[2] - pb[2]};
                    for (int r = 0; r < 3; ++r) b[r] = Rb[r] * d[0] + Rb[3 + r] * d[1] + Rb[6 + r] * d[2];
                }
                if (dep > 0.0 && nc < OR_MAXFC) {
                    memcpy(cw[nc], x, sizeof x);
                    memcpy(cb[nc], b, sizeof b);
                    depth[nc] = dep;
                    cbody[nc] = bi;
                    cslot[nc] = slot_id;
                    ++nc;
                }
            }
        }
    }

    /* rows: J, rhs, bounds kind */
    enum { K_NORMAL, K_FRIC, K_BOX };
    static _Thread_local double J[3 * OR_MAXFC + 3 * OR_MAXB][6 + OR_MAXB];
    static _Thread_local double MJ[3 * OR_MAXFC + 3 * OR_MAXB][6 + OR_MAXB];
    static _Thread_local double A[(3 * OR_MAXFC + 3 * OR_MAXB) * (3 * OR_MAXFC + 3 * OR_MAXB)];
    double bb[3 * OR_MAXFC + 3 * OR_MAXB], lo[3 * OR_MAXFC + 3 * OR_MAXB], hi[3 * OR_MAXFC + 3 * OR_MAXB];
    double cfm[3 * OR_MAXFC + 3 * OR_MAXB], x[3 * OR_MAXFC + 3 * OR_MAXB];
    double bsc[3 * OR_MAXFC + 3 * OR_MAXB];
    int kind[3 * OR_MAXFC + 3 * OR_MAXB];
    int wid[3 * OR_MAXFC + 3 * OR_MAXB];
    int nr = 0;
    const double nrm[3] = {0, 0, 1};
    double t1[3], t2[3];
    plane_space(nrm, t1, t2);
    for (int c = 0; c < nc; ++c) {
        const int bi = cbody[c];
        const double* Rb = bi < 0 ? s->R : k.Rw[bi];
        for (int d = 0; d < 3; ++d) {
            const double* dw = d == 0 ? nrm : (d == 1 ? t1 : t2);
            double f[6];
            for (int r = 0; r < 3; ++r) f[3 + r] = Rb[r] * dw[0] + Rb[3 + r] * dw[1] + Rb[6 + r] * dw[2];
            cross3(cb[c], f + 3, f);
            if (bi < 0) {
                for (int e = 0; e < nv; ++e) J[nr][e] = 0.0;
                for (int e = 0; e < 6; ++e) J[nr][e] = f[e];
            } else {
                float_row(m, &k, bi, f, J[nr]);
            }
            double vrel = 0.0, vabs = 0.0;
            for (int e = 0; e < nv; ++e) {
                vrel += J[nr][e] * nu[e];
                vabs += fabs(J[nr][e] * nu[e]);
            }
            double bounce = 0.0;
            if (d == 0) {
                bounce = OR_C_ERP * depth[c] / dt;
                if (bounce > OR_C_MAX_ERV) bounce = OR_C_MAX_ERV;
            }
            bb[nr] = -vrel + bounce;
            bsc[nr] = vabs + bounce;
            kind[nr] = d == 0 ? K_NORMAL : K_FRIC;
            cfm[nr] = OR_C_CFM;
            wid[nr] = 3 * cslot[c] + d;
            ++nr;
        }
    }
    for (int i = 0; i < n; ++i) {
        const double qdi = nu[6 + i];
        int rows_i[3], nri = 0;
        if (t->limited[i]) {
            double viol = s->q[i] - t->lower[i];
            int active = 0;
            if (viol <= 0.0) { lo[nr] = 0.0; hi[nr] = INFINITY; active = 1; }
            else {
                viol = s->q[i] - t->upper[i];
                if (viol >= 0.0) { lo[nr] = -INFINITY; hi[nr] = 0.0; active = 1; }
            }
            if (active) {
                double bounce = -viol * OR_ERP / dt;
                if (bounce > OR_MAX_ERV) bounce = OR_MAX_ERV;
                if (bounce < -OR_MAX_ERV) bounce = -OR_MAX_ERV;
                bb[nr] = -qdi + bounce;
                bsc[nr] = fabs(qdi) + fabs(bounce);
                wid[nr] = OR_WARM_JOINT0 + 3 * i;
                rows_i[nri++] = nr++;
            }
        }
        if (mode[i] == OR_SERVO) {
            double vc = cmd[i];
            if (vc < -t->vel_limit[i]) vc = -t->vel_limit[i];
            if (vc > t->vel_limit[i]) vc = t->vel_limit[i];
            if (vc - qdi != 0.0) {
                bb[nr] = vc - qdi;
                bsc[nr] = fabs(vc) + fabs(qdi);
                lo[nr] = -t->effort[i] * dt;
                hi[nr] = t->effort[i] * dt;
                wid[nr] = OR_WARM_JOINT0 + 3 * i + 1;
                rows_i[nri++] = nr++;
            }
        }
        if (t->friction[i] != 0.0 && qdi != 0.0) {
            bb[nr] = -qdi;
            bsc[nr] = fabs(qdi);
            hi[nr] = t->friction[i] * dt;
            lo[nr] = -hi[nr];
            wid[nr] = OR_WARM_JOINT0 + 3 * i + 2;
            rows_i[nri++] = nr++;
        }
        for (int r = 0; r < nri; ++r) {
            const int row = rows_i[r];
            for (int e = 0; e < nv; ++e) J[row][e] = 0.0;
            J[row][6 + i] = 1.0;
            kind[row] = K_BOX;
            cfm[row] = OR_CFM;
        }
    }
    if (nr > 0) {
        for (int r = 0; r < nr; ++r) solve_dense(nv, M, J[r], MJ[r]);
        for (int r = 0; r < nr; ++r) {
            for (int c = 0; c < nr; ++c) {
                double a = 0.0;
                for (int e = 0; e < nv; ++e) a += J[r][e] * MJ[c][e];
                A[r * nr + c] = a;
            }
            A[r * nr + r] *= 1.0 + cfm[r];
            x[r] = warm ? warm[wid[r]] : 0.0;
        }
        g_cap_n = nr;
        g_cap_mu = m->mu;
        for (int r = 0; r < nr; ++r) {
            for (int c = 0; c < nr; ++c) g_cap_A[r * nr + c] = A[r * nr + c];
            g_cap_b[r] = bb[r];
            g_cap_wid[r] = wid[r];
            g_cap_bscale[r] = bsc[r];
            g_cap_x1[r] = 0.0;
            g_cap_kind[r] = kind[r];
            g_cap_lo[r] = kind[r] == K_BOX ? lo[r] : (kind[r] == K_NORMAL ? 0.0 : -INFINITY);
            g_cap_hi[r] = kind[r] == K_BOX ? hi[r] : INFINITY;
        }
        g_pgs_sweeps = 0;
        for (int it = 0; it < pgs_budget(pgs_iters); ++it) {
            double x_start[3 * OR_MAXFC + 3 * OR_MAXB];
            memcpy(x_start, x, sizeof(double) * (size_t)nr);
            for (int r = 0; r < nr; ++r) {
                double acc_r = bb[r];
                for (int c = 0; c < nr; ++c) acc_r -= A[r * nr + c] * x[c];
                double v = x[r] + acc_r / A[r * nr + r];
                double l = lo[r], u = hi[r];
                if (kind[r] == K_NORMAL) { l = 0.0; u = INFINITY; }
                else if (kind[r] == K_FRIC) {
                    const int nrow = r - (r % 3);
                    u = m->mu * x[nrow];
                    l = -u;
                }
                if (v < l) v = l;
                if (v > u) v = u;
                x[r] = v;
            }
            pgs_count(it);
            /* tolerance exit (the kernels' pgs_tol): the sweep changed no row's
             * constraint velocity (A x)_r by more than pgs_tol */
            if (pgs_tol > 0.0 && pgs_iters >= 0) {
                double dmax = 0.0;
                for (int r = 0; r < nr; ++r) {
                    double dw = 0.0;
                    for (int c = 0; c < nr; ++c) dw += A[r * nr + c] * (x[c] - x_start[c]);
                    if (fabs(dw) > dmax) dmax = fabs(dw);
                }
                if (dmax <= pgs_tol) break;
            }
        }
        if (pgs_iters < 0) {
            int findex[3 * OR_MAXFC + 3 * OR_MAXB];
            for (int r = 0; r < nr; ++r) {
                findex[r] = (kind[r] == K_FRIC) ? r - (r % 3) : -1;
                if (kind[r] == K_NORMAL) { lo[r] = 0.0; hi[r] = INFINITY; }
            }
            lcp_dantzig(nr, A, nr, bb, lo, hi, findex, m->mu, x);
            for (int r = 0; r < nr; ++r) g_cap_x1[r] = g_last_x1[r];
        }
        for (int r = 0; r < nr; ++r) g_cap_x[r] = x[r];
        for (int r = 0; r < nr; ++r)
            for (int e = 0; e < nv; ++e) nu[e] += MJ[r][e] * x[r];
    }
    if (warm) {
        for (int e = 0; e < OR_WARM_WORDS; ++e) warm[e] = 0.0;
        for (int r = 0; r < nr; ++r) warm[wid[r]] = x[r];
    }

    /* integratePositions: q += dt qd; T0 <- T0 exp(dt V0) */
    for (int i = 0; i < n; ++i) s->qd[i] = nu[6 + i];
    integrate_joint_positions(t, s->q, s->qd, dt);
    double phi[3] = {dt * nu[0], dt * nu[1], dt * nu[2]}, u[3] = {dt * nu[3], dt * nu[4], dt * nu[5]};
    double dR[9], dp[3], Rn[9];
    se3_exp(phi, u, dR, dp);
    for (int r = 0; r < 3; ++r) {
        s->p[r] += s->R[r * 3] * dp[0] + s->R[r * 3 + 1] * dp[1] + s->R[r * 3 + 2] * dp[2];
        for (int q = 0; q < 3; ++q)
            Rn[r * 3 + q] = s->R[r * 3] * dR[q] + s->R[r * 3 + 1] * dR[3 + q] + s->R[r * 3 + 2] * dR[6 + q];
    }
    memcpy(s->R, Rn, sizeof Rn);
    for (int e = 0; e < 6; ++e) s->V[e] = nu[e];

    for (int c = 0; c < nc; ++c) {
        for (int r = 0; r < 3; ++r) {
            if (c_pos) c_pos[3 * c + r] = cw[c][r];
            if (c_force) c_force[3 * c + r] = (nrm[r] * x[3 * c] + t1[r] * x[3 * c + 1] + t2[r] * x[3 * c + 2]) / dt;
        }
        if (c_depth) c_depth[c] = depth[c];
        if (c_body) c_body[c] = cbody[c];
    }
    return nc;
}

/* ====================================================================== */
/* Scene: several models in one world, shape-pair contacts, wrenches.     */
/* ====================================================================== */

static double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

/* column k of a row-major rotation (the k-th shape axis in the world) */
static void col3(const double* R, int k, double out[3])
{
    out[0] = R[k]; out[1] = R[3 + k]; out[2] = R[6 + k];
}

/* reduce n > 4 contact points to 4 (deterministic): the deepest, the one
 * farthest from it, the one farthest from the line through both, then the
 * one farthest from the triangle's plane-projected centroid */
static int reduce_points(int n, double (*p)[3], double* d)
{
    if (n <= 4) return n;
    int keep[4], used[8] = {0};
    int a = 0;
    for (int i = 1; i < n; ++i) if (d[i] > d[a]) a = i;
    keep[0] = a; used[a] = 1;
    int b = -1; double best = -1.0;
    for (int i = 0; i < n; ++i) {
        if (used[i]) continue;
        double e[3] = {p[i][0] - p[a][0], p[i][1] - p[a][1], p[i][2] - p[a][2]};
        const double v = dot3(e, e);
        if (v > best) { best = v; b = i; }
    }
    keep[1] = b; used[b] = 1;
    int c = -1; best = -1.0;
    const double ab[3] = {p[b][0] - p[a][0], p[b][1] - p[a][1], p[b][2] - p[a][2]};
    for (int i = 0; i < n; ++i) {
        if (used[i]) continue;
        double e[3] = {p[i][0] - p[a][0], p[i][1] - p[a][1], p[i][2] - p[a][2]}, x[3];
        cross3(ab, e, x);
        const double v = dot3(x, x);
        if (v > best) { best = v; c = i; }
    }
    keep[2] = c; used[c] = 1;
    int e4 = -1; best = -1.0;
    const double g[3] = {(p[a][0] + p[b][0] + p[c][0]) / 3.0, (p[a][1] + p[b][1] + p[c][1]) / 3.0,
                         (p[a][2] + p[b][2] + p[c][2]) / 3.0};
    for (int i = 0; i < n; ++i) {
        if (used[i]) continue;
        double e[3] = {p[i][0] - g[0], p[i][1] - g[1], p[i][2] - g[2]};
        const double v = dot3(e, e);
        if (v > best) { best = v; e4 = i; }
    }
    keep[3] = e4;
    /* keep the original order of the survivors */
    double tp[4][3], td[4];
    int m = 0;
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < 4; ++k)
            if (keep[k] == i) { memcpy(tp[m], p[i], sizeof tp[m]); td[m] = d[i]; ++m; }
    for (int i = 0; i < 4; ++i) { memcpy(p[i], tp[i], sizeof tp[i]); d[i] = td[i]; }
    return 4;
}

/* Sutherland-Hodgman clip of a polygon (2D coordinates in (u, v) plus the 3D
 * point) against |u| <= hu, |v| <= hv */
static int clip_polygon(int n, double (*poly)[5], double hu, double hv, double (*out)[5])
{
    double buf[2][16][5];
    int cnt = n;
    memcpy(buf[0], poly, (size_t)n * sizeof(double[5]));
    int cur = 0;
    for (int plane = 0; plane < 4; ++plane) {
        const int axis = plane >> 1;              /* 0: u, 1: v */
        const double sg = (plane & 1) ? -1.0 : 1.0; /* keep sg * x <= h */
        const double h = axis ? hv : hu;
        int m = 0;
        double (*src)[5] = buf[cur], (*dst)[5] = buf[cur ^ 1];
        for (int i = 0; i < cnt; ++i) {
            const double* P = src[i];
            const double* Q = src[(i + 1) % cnt];
            const double dp = sg * P[axis] - h, dq = sg * Q[axis] - h;
            if (dp <= 0.0) { memcpy(dst[m++], P, sizeof(double[5])); }
            if ((dp < 0.0 && dq > 0.0) || (dp > 0.0 && dq < 0.0)) {
                const double t = dp / (dp - dq);
                for (int k = 0; k < 5; ++k) dst[m][k] = P[k] + t * (Q[k] - P[k]);
                ++m;
            }
        }
        cnt = m;
        cur ^= 1;
        if (cnt == 0) return 0;
    }
    memcpy(out, buf[cur], (size_t)cnt * sizeof(double[5]));
    return cnt;
}

static int box_box(const double* hA, const double* cA, const double* RA, const double* hB, const double* cB,
                   const double* RB, double n[3], double* pts, double* deps)
{
    double a[3][3], b[3][3], T[3] = {cB[0] - cA[0], cB[1] - cA[1], cB[2] - cA[2]};
    for (int k = 0; k < 3; ++k) { col3(RA, k, a[k]); col3(RB, k, b[k]); }
    /* face axes: k < 3 of A, 3..5 of B */
    double best_face = INFINITY, best_edge = INFINITY;
    int face = -1, ei = -1, ej = -1;
    double edge_axis[3] = {0, 0, 0};
    for (int k = 0; k < 6; ++k) {
        const double* L = k < 3 ? a[k] : b[k - 3];
        double rA = 0.0, rB = 0.0;
        for (int i = 0; i < 3; ++i) { rA += hA[i] * fabs(dot3(a[i], L)); rB += hB[i] * fabs(dot3(b[i], L)); }
        const double pen = rA + rB - fabs(dot3(T, L));
        if (pen < 0.0) return 0;
        if (pen < best_face) { best_face = pen; face = k; }
    }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double L[3];
            cross3(a[i], b[j], L);
            const double len = sqrt(dot3(L, L));
            if (len < 1e-6) continue;
            for (int k = 0; k < 3; ++k) L[k] /= len;
            double rA = 0.0, rB = 0.0;
            for (int k = 0; k < 3; ++k) { rA += hA[k] * fabs(dot3(a[k], L)); rB += hB[k] * fabs(dot3(b[k], L)); }
            const double pen = rA + rB - fabs(dot3(T, L));
            if (pen < 0.0) return 0;
            if (pen < best_edge) { best_edge = pen; ei = i; ej = j; memcpy(edge_axis, L, sizeof L); }
        }
    /* face contacts unless an edge axis is clearly shallower */
    if (ei >= 0 && best_edge < 0.95 * best_face - 1e-5) {
        double L[3] = {edge_axis[0], edge_axis[1], edge_axis[2]};
        if (dot3(L, T) > 0.0) for (int k = 0; k < 3; ++k) L[k] = -L[k];   /* from B to A */
        memcpy(n, L, sizeof L);
        /* the edge of A nearest B (direction -n) and of B nearest A (+n) */
        double pa[3], pb[3];
        memcpy(pa, cA, sizeof pa);
        memcpy(pb, cB, sizeof pb);
        for (int k = 0; k < 3; ++k) {
            if (k != ei) {
                const double sg = dot3(a[k], n) > 0.0 ? -1.0 : 1.0;
                for (int r = 0; r < 3; ++r) pa[r] += sg * hA[k] * a[k][r];
            }
            if (k != ej) {
                const double sg = dot3(b[k], n) > 0.0 ? 1.0 : -1.0;
                for (int r = 0; r < 3; ++r) pb[r] += sg * hB[k] * b[k][r];
            }
        }
        /* closest points of the two edge lines, clamped to the edges */
        const double* u = a[ei];
        const double* v = b[ej];
        double w0[3] = {pa[0] - pb[0], pa[1] - pb[1], pa[2] - pb[2]};
        const double uv = dot3(u, v), uw = dot3(u, w0), vw = dot3(v, w0);
        const double den = 1.0 - uv * uv;
        double s = den > 1e-12 ? (uv * vw - uw) / den : 0.0;
        double t = den > 1e-12 ? (vw - uv * uw) / den : 0.0;
        if (s < -hA[ei]) s = -hA[ei];
        if (s > hA[ei]) s = hA[ei];
        if (t < -hB[ej]) t = -hB[ej];
        if (t > hB[ej]) t = hB[ej];
        for (int r = 0; r < 3; ++r) pts[r] = 0.5 * (pa[r] + s * u[r] + pb[r] + t * v[r]);
        deps[0] = best_edge;
        return 1;
    }
    /* face case: reference box owns the axis, incident box is the other */
    const int refA = face < 3;
    const int fk = refA ? face : face - 3;
    const double* cR = refA ? cA : cB;
    const double* cI = refA ? cB : cA;
    const double* hR = refA ? hA : hB;
    const double* hI = refA ? hB : hA;
    double (*R)[3] = refA ? a : b;
    double (*I)[3] = refA ? b : a;
    double nr[3];   /* reference face normal, pointing towards the incident box */
    memcpy(nr, R[fk], sizeof nr);
    const double tI[3] = {cI[0] - cR[0], cI[1] - cR[1], cI[2] - cR[2]};
    if (dot3(nr, tI) < 0.0) for (int k = 0; k < 3; ++k) nr[k] = -nr[k];
    /* n from B to A: the reference normal points from R to I */
    for (int k = 0; k < 3; ++k) n[k] = refA ? -nr[k] : nr[k];
    /* incident face: most anti-parallel to nr */
    int ik = 0;
    double bd = 0.0;
    for (int k = 0; k < 3; ++k) {
        const double d = fabs(dot3(I[k], nr));
        if (d > bd) { bd = d; ik = k; }
    }
    const double sg = dot3(I[ik], nr) > 0.0 ? -1.0 : 1.0;
    const int k1 = (ik + 1) % 3, k2 = (ik + 2) % 3;
    const int u1 = (fk + 1) % 3, u2 = (fk + 2) % 3;
    double fc[3];   /* reference face centre */
    for (int r = 0; r < 3; ++r) fc[r] = cR[r] + hR[fk] * nr[r];
    double poly[4][5];
    const double sx[4] = {1, -1, -1, 1}, sy[4] = {1, 1, -1, -1};
    for (int q = 0; q < 4; ++q) {
        double x[3];
        for (int r = 0; r < 3; ++r)
            x[r] = cI[r] + sg * hI[ik] * I[ik][r] + sx[q] * hI[k1] * I[k1][r] + sy[q] * hI[k2] * I[k2][r];
        const double rel[3] = {x[0] - fc[0], x[1] - fc[1], x[2] - fc[2]};
        poly[q][0] = dot3(rel, R[u1]);
        poly[q][1] = dot3(rel, R[u2]);
        poly[q][2] = x[0]; poly[q][3] = x[1]; poly[q][4] = x[2];
    }
    double clipped[16][5];
    const int m = clip_polygon(4, poly, hR[u1], hR[u2], clipped);
    double P[16][3], D[16];
    int cnt = 0;
    for (int i = 0; i < m; ++i) {
        const double* x = clipped[i] + 2;
        const double rel[3] = {fc[0] - x[0], fc[1] - x[1], fc[2] - x[2]};
        const double dep = dot3(rel, nr);
        if (dep > 0.0 && cnt < 8) {
            memcpy(P[cnt], x, sizeof P[cnt]);
            D[cnt] = dep;
            ++cnt;
        }
    }
    cnt = reduce_points(cnt, P, D);
    for (int i = 0; i < cnt; ++i) { memcpy(pts + 3 * i, P[i], sizeof P[i]); deps[i] = D[i]; }
    return cnt;
}

/* box (A or B) against a sphere; nbs: unit normal from the box into the
 * sphere; the point lies on the box surface */
static int box_sphere(const double* h, const double* c, const double* R, double rad, const double* s,
                      double nbs[3], double* pt, double* dep)
{
    const double d[3] = {s[0] - c[0], s[1] - c[1], s[2] - c[2]};
    double l[3], q[3];
    int inside = 1;
    for (int k = 0; k < 3; ++k) {
        l[k] = R[k] * d[0] + R[3 + k] * d[1] + R[6 + k] * d[2];
        q[k] = l[k] < -h[k] ? -h[k] : (l[k] > h[k] ? h[k] : l[k]);
        if (q[k] != l[k]) inside = 0;
    }
    if (!inside) {
        double e[3] = {l[0] - q[0], l[1] - q[1], l[2] - q[2]};
        const double dist = sqrt(dot3(e, e));
        if (dist > rad) return 0;
        for (int k = 0; k < 3; ++k) e[k] /= dist;
        for (int r = 0; r < 3; ++r) {
            nbs[r] = R[r * 3] * e[0] + R[r * 3 + 1] * e[1] + R[r * 3 + 2] * e[2];
            pt[r] = c[r] + R[r * 3] * q[0] + R[r * 3 + 1] * q[1] + R[r * 3 + 2] * q[2];
        }
        *dep = rad - dist;
        return 1;
    }
    int kk = 0;
    double best = INFINITY;
    for (int k = 0; k < 3; ++k) {
        const double g = h[k] - fabs(l[k]);
        if (g < best) { best = g; kk = k; }
    }
    const double sg = l[kk] >= 0.0 ? 1.0 : -1.0;
    double lq[3] = {l[0], l[1], l[2]};
    lq[kk] = sg * h[kk];
    for (int r = 0; r < 3; ++r) {
        nbs[r] = sg * R[r * 3 + kk];
        pt[r] = c[r] + R[r * 3] * lq[0] + R[r * 3 + 1] * lq[1] + R[r * 3 + 2] * lq[2];
    }
    *dep = rad + best;
    return 1;
}

/* cylinder (h = {radius, half length}, axis = local z) against a sphere;
 * same conventions as box_sphere: nbs from the cylinder into the sphere, the
 * point on the cylinder surface.  Outside: the closest point of the solid
 * cylinder; centre inside: the nearest of the side and the two caps. */
static int cylinder_sphere(const double* h, const double* c, const double* R, double rad, const double* s,
                           double nbs[3], double* pt, double* dep)
{
    const double d[3] = {s[0] - c[0], s[1] - c[1], s[2] - c[2]};
    double l[3], q[3];
    for (int k = 0; k < 3; ++k) l[k] = R[k] * d[0] + R[3 + k] * d[1] + R[6 + k] * d[2];
    const double rho = sqrt(l[0] * l[0] + l[1] * l[1]);
    const int inside = rho <= h[0] && fabs(l[2]) <= h[1];
    if (!inside) {
        const double k = rho > h[0] ? h[0] / rho : 1.0;
        q[0] = l[0] * k;
        q[1] = l[1] * k;
        q[2] = l[2] < -h[1] ? -h[1] : (l[2] > h[1] ? h[1] : l[2]);
        double e[3] = {l[0] - q[0], l[1] - q[1], l[2] - q[2]};
        const double dist = sqrt(dot3(e, e));
        if (dist > rad || dist == 0.0) return 0;
        for (int k2 = 0; k2 < 3; ++k2) e[k2] /= dist;
        for (int r = 0; r < 3; ++r) {
            nbs[r] = R[r * 3] * e[0] + R[r * 3 + 1] * e[1] + R[r * 3 + 2] * e[2];
            pt[r] = c[r] + R[r * 3] * q[0] + R[r * 3 + 1] * q[1] + R[r * 3 + 2] * q[2];
        }
        *dep = rad - dist;
        return 1;
    }
    const double gs = h[0] - rho, gc = h[1] - fabs(l[2]);
    double e[3];
    if (gs < gc && rho > 0.0) {   /* through the side */
        e[0] = l[0] / rho; e[1] = l[1] / rho; e[2] = 0.0;
        q[0] = h[0] * e[0]; q[1] = h[0] * e[1]; q[2] = l[2];
        *dep = rad + gs;
    } else {                      /* through a cap */
        const double sg = l[2] >= 0.0 ? 1.0 : -1.0;
        e[0] = 0.0; e[1] = 0.0; e[2] = sg;
        q[0] = l[0]; q[1] = l[1]; q[2] = sg * h[1];
        *dep = rad + gc;
    }
    for (int r = 0; r < 3; ++r) {
        nbs[r] = R[r * 3] * e[0] + R[r * 3 + 1] * e[1] + R[r * 3 + 2] * e[2];
        pt[r] = c[r] + R[r * 3] * q[0] + R[r * 3 + 1] * q[1] + R[r * 3 + 2] * q[2];
    }
    return 1;
}

/* 8 sample points of a box / cylinder for the cylinder-pair narrow phase
 * (see cylinder_pair) */
static void pair_samples(int type, const double* h, const double* c, const double* R, const double* other,
                         double out[8][3])
{
    for (int k = 0; k < 8; ++k) {
        double l[3];
        if (type == 0) {
            l[0] = (k & 4) ? h[0] : -h[0];
            l[1] = (k & 2) ? h[1] : -h[1];
            l[2] = (k & 1) ? h[2] : -h[2];
        } else {
            const double d[3] = {other[0] - c[0], other[1] - c[1], other[2] - c[2]};
            double ux = R[0] * d[0] + R[3] * d[1] + R[6] * d[2], uy = R[1] * d[0] + R[4] * d[1] + R[7] * d[2];
            const double n2 = ux * ux + uy * uy;
            if (n2 > 1e-12) {
                const double inv = 1.0 / sqrt(n2);
                ux *= inv;
                uy *= inv;
            } else {
                ux = 1.0;
                uy = 0.0;
            }
            const int j = k & 3;
            const double dx = (j == 0) ? ux : ((j == 1) ? -uy : ((j == 2) ? -ux : uy));
            const double dy = (j == 0) ? uy : ((j == 1) ? ux : ((j == 2) ? -uy : -ux));
            l[0] = 0.999 * h[0] * dx;
            l[1] = 0.999 * h[0] * dy;
            l[2] = (k & 4) ? h[1] : -h[1];
        }
        for (int r = 0; r < 3; ++r) out[k][r] = c[r] + R[r * 3] * l[0] + R[r * 3 + 1] * l[1] + R[r * 3 + 2] * l[2];
    }
}

/* point p inside shape (box / cylinder)?  outward normal at the nearest face, depth */
static int inside_shape(int type, const double* h, const double* c, const double* R, const double* p, double n[3],
                        double* dep)
{
    const double d[3] = {p[0] - c[0], p[1] - c[1], p[2] - c[2]};
    double l[3], e[3] = {0.0, 0.0, 0.0};
    for (int k = 0; k < 3; ++k) l[k] = R[k] * d[0] + R[3 + k] * d[1] + R[6 + k] * d[2];
    if (type == 0) {
        int best = -1;
        double pen = 0.0;
        for (int k = 0; k < 3; ++k) {
            const double g = h[k] - fabs(l[k]);
            if (g <= 0.0) return 0;
            if (best < 0 || g < pen) { pen = g; best = k; }
        }
        e[best] = l[best] >= 0.0 ? 1.0 : -1.0;
        *dep = pen;
    } else {
        const double rho = sqrt(l[0] * l[0] + l[1] * l[1]);
        const double gs = h[0] - rho, gc = h[1] - fabs(l[2]);
        if (gs <= 0.0 || gc <= 0.0) return 0;
        if (gs < gc && rho > 0.0) {
            e[0] = l[0] / rho;
            e[1] = l[1] / rho;
            *dep = gs;
        } else {
            e[2] = l[2] >= 0.0 ? 1.0 : -1.0;
            *dep = gc;
        }
    }
    for (int r = 0; r < 3; ++r) n[r] = R[r * 3] * e[0] + R[r * 3 + 1] * e[1] + R[r * 3 + 2] * e[2];
    return 1;
}

/* support extent of a box / cylinder along the unit direction n */
static double shape_support(int type, const double* h, const double* R, const double* n)
{
    if (type == 0) {
        double s = 0.0;
        for (int k = 0; k < 3; ++k) s += h[k] * fabs(n[0] * R[k] + n[1] * R[3 + k] + n[2] * R[6 + k]);
        return s;
    }
    const double c = n[0] * R[2] + n[1] * R[5] + n[2] * R[8];
    const double s2 = 1.0 - c * c;
    return h[0] * sqrt(s2 > 0.0 ? s2 : 0.0) + h[1] * fabs(c);
}

/* candidate separating axes of one shape: box face normals; cylinder axis
 * and the radial direction towards the other shape's centre */
static int shape_axes(int type, const double* c, const double* R, const double* other, double ax[3][3])
{
    if (type == 0) {
        for (int k = 0; k < 3; ++k) col3(R, k, ax[k]);
        return 3;
    }
    col3(R, 2, ax[0]);
    const double d[3] = {other[0] - c[0], other[1] - c[1], other[2] - c[2]};
    const double t = dot3(d, ax[0]);
    double q[3] = {d[0] - t * ax[0][0], d[1] - t * ax[0][1], d[2] - t * ax[0][2]};
    const double nq = sqrt(dot3(q, q));
    if (nq <= 1e-9) return 1;
    for (int k = 0; k < 3; ++k) ax[1][k] = q[k] / nq;
    return 2;
}

/* Cylinder pairs (cylinder-box, cylinder-cylinder; DART's collision detector
 * [EXT] works on the exact geometry): the contact normal is the candidate
 * axis of least overlap (supports of both shapes minus the centre distance
 * along it; A's axes then B's, first on ties; no overlap on some axis = no
 * contact), oriented from B into A.  The points are sampled features: 8 per
 * shape -- a box's corners, a cylinder's 4 rim points per cap at 0.999 r,
 * 90 degrees apart, the first facing the other shape's centre (x axis when
 * coaxial) -- that lie inside the other shape and beyond its extreme plane
 * along the normal (depth = distance past that plane); A's samples then B's,
 * at most 8, reduced to 4 by reduce_points. */
static int cylinder_pair(int ta, const double* ha, const double* ca, const double* Ra, int tb, const double* hb,
                         const double* cb, const double* Rb, double normal[3], double* points, double* depths)
{
    double ax[6][3];
    int na = shape_axes(ta, ca, Ra, cb, ax);
    na += shape_axes(tb, cb, Rb, ca, ax + na);
    const double dab[3] = {ca[0] - cb[0], ca[1] - cb[1], ca[2] - cb[2]};
    int best = -1;
    double ov_min = 0.0;
    for (int k = 0; k < na; ++k) {
        const double ov = shape_support(ta, ha, Ra, ax[k]) + shape_support(tb, hb, Rb, ax[k]) - fabs(dot3(ax[k], dab));
        if (ov <= 0.0) return 0;
        if (best < 0 || ov < ov_min) { ov_min = ov; best = k; }
    }
    double n[3];
    const double sg = dot3(ax[best], dab) >= 0.0 ? 1.0 : -1.0;
    for (int k = 0; k < 3; ++k) n[k] = sg * ax[best][k];
    const double plane_b = dot3(n, cb) + shape_support(tb, hb, Rb, n);   /* B's face towards A */
    const double plane_a = dot3(n, ca) - shape_support(ta, ha, Ra, n);   /* A's face towards B */
    double sp[2][8][3];
    pair_samples(ta, ha, ca, Ra, cb, sp[0]);
    pair_samples(tb, hb, cb, Rb, ca, sp[1]);
    double p[8][3], d[8];
    int m = 0;
    for (int side = 0; side < 2; ++side)
        for (int k = 0; k < 8 && m < 8; ++k) {
            double nn[3], dd;
            const int in = side ? inside_shape(ta, ha, ca, Ra, sp[1][k], nn, &dd)
                                : inside_shape(tb, hb, cb, Rb, sp[0][k], nn, &dd);
            const double dep = side ? dot3(n, sp[1][k]) - plane_a : plane_b - dot3(n, sp[0][k]);
            if (!in || dep <= 0.0) continue;
            memcpy(p[m], sp[side][k], sizeof p[m]);
            d[m] = dep;
            ++m;
        }
    m = reduce_points(m, p, d);
    memcpy(normal, n, sizeof n);
    for (int i = 0; i < m; ++i) {
        memcpy(points + 3 * i, p[i], 3 * sizeof(double));
        depths[i] = d[i];
    }
    return m;
}

/* world point of a shape-frame point: c + R v (R row-major) */
static void mat_vec3(const double* R, const double* v, const double* c, double* out)
{
    for (int r = 0; r < 3; ++r) out[r] = c[r] + R[3 * r] * v[0] + R[3 * r + 1] * v[1] + R[3 * r + 2] * v[2];
}

static void rot3(const double* R, const double* v, double* out)
{
    for (int r = 0; r < 3; ++r) out[r] = R[3 * r] * v[0] + R[3 * r + 1] * v[1] + R[3 * r + 2] * v[2];
}

/* ---------------- convex hulls of mesh shapes (narrow phase) ----------------
 * The reference attaches a <mesh> collision to DART as its triangle mesh
 * (Physics.cpp:897-931) [EXT].  Restated here as the convex hull of the mesh
 * shape's support points (the same <= OR_MESH_MAXP hull vertices that touch
 * the ground plane; a mesh with at most that many hull vertices gets its
 * exact hull), colliding with boxes and other meshes by the separating-axis
 * test over face normals and edge-pair directions, with the reference face
 * clipped against the incident face as box_box does (round 6: replaces the
 * bounding-box stand-in).  Built in fp64 by brute force: a face is a plane
 * through three points with every point on its inner side; coplanar points
 * share one polygon face, ordered counter-clockwise seen from outside. */
typedef struct {
    int nv, nf, ne;
    double v[OR_MESH_MAXP][3];
    double n[OR_HULL_MAXF][3];
    double d[OR_HULL_MAXF];                 /* inside: n . x <= d */
    int fnv[OR_HULL_MAXF];
    int fv[OR_HULL_MAXF][OR_MESH_MAXP];
    int e[OR_HULL_MAXE][2];
    int ef[OR_HULL_MAXE][2];                /* the two faces meeting at each edge */
    double ctr[3];                          /* vertex centroid (interior) */
} or_hull;

static int or_hull_make(int np, const double* pts, or_hull* h)
{
    memset(h, 0, sizeof *h);
    if (np > OR_MESH_MAXP) np = OR_MESH_MAXP;
    h->nv = np;
    double scale = 0.0;
    for (int i = 0; i < np; ++i)
        for (int k = 0; k < 3; ++k) {
            h->v[i][k] = pts[3 * i + k];
            h->ctr[k] += pts[3 * i + k] / np;
            scale = fabs(pts[3 * i + k]) > scale ? fabs(pts[3 * i + k]) : scale;
        }
    const double eps = 1e-9 * (scale > 0.0 ? scale : 1.0);
    for (int i = 0; i < np; ++i)
        for (int j = i + 1; j < np; ++j)
            for (int k = j + 1; k < np; ++k) {
                double a[3], b[3], n[3];
                for (int q = 0; q < 3; ++q) { a[q] = h->v[j][q] - h->v[i][q]; b[q] = h->v[k][q] - h->v[i][q]; }
                cross3(a, b, n);
                const double len = sqrt(dot3(n, n));
                if (len <= 1e-12 * (scale * scale > 0.0 ? scale * scale : 1.0)) continue;   /* collinear */
                for (int q = 0; q < 3; ++q) n[q] /= len;
                double d = dot3(n, h->v[i]), hi = -INFINITY, lo = INFINITY;
                for (int m = 0; m < np; ++m) {
                    const double s = dot3(n, h->v[m]) - d;
                    hi = s > hi ? s : hi;
                    lo = s < lo ? s : lo;
                }
                if (hi > eps && lo < -eps) continue;      /* points on both sides: not a face */
                if (hi > eps) {                          /* all above: the outward normal is -n */
                    for (int q = 0; q < 3; ++q) n[q] = -n[q];
                    d = -d;
                }
                int dup = 0;
                for (int f = 0; f < h->nf && !dup; ++f)
                    dup = fabs(dot3(h->n[f], n) - 1.0) < 1e-9 && fabs(h->d[f] - d) <= 4 * eps;
                if (dup || h->nf >= OR_HULL_MAXF) continue;
                const int f = h->nf++;
                memcpy(h->n[f], n, sizeof n);
                h->d[f] = d;
            }
    if (h->nf < 4) return 0;   /* flat or degenerate point set: no volume */
    /* face polygons: the points on each plane, counter-clockwise about n */
    for (int f = 0; f < h->nf; ++f) {
        double c[3] = {0, 0, 0}, u[3], w[3], ang[OR_MESH_MAXP];
        int idx[OR_MESH_MAXP], m = 0;
        for (int i = 0; i < np; ++i)
            if (fabs(dot3(h->n[f], h->v[i]) - h->d[f]) <= 4 * eps) idx[m++] = i;
        for (int t = 0; t < m; ++t)
            for (int q = 0; q < 3; ++q) c[q] += h->v[idx[t]][q] / m;
        for (int q = 0; q < 3; ++q) u[q] = h->v[idx[0]][q] - c[q];
        const double ul = sqrt(dot3(u, u));
        for (int q = 0; q < 3; ++q) u[q] /= ul;
        cross3(h->n[f], u, w);
        for (int t = 0; t < m; ++t) {
            double r[3] = {h->v[idx[t]][0] - c[0], h->v[idx[t]][1] - c[1], h->v[idx[t]][2] - c[2]};
            ang[t] = atan2(dot3(r, w), dot3(r, u));
        }
        for (int a = 1; a < m; ++a)        /* insertion sort by angle */
            for (int b = a; b > 0 && ang[b] < ang[b - 1]; --b) {
                const double ta = ang[b]; ang[b] = ang[b - 1]; ang[b - 1] = ta;
                const int ti = idx[b]; idx[b] = idx[b - 1]; idx[b - 1] = ti;
            }
        h->fnv[f] = m;
        for (int t = 0; t < m; ++t) h->fv[f][t] = idx[t];
        for (int t = 0; t < m; ++t) {
            int a = idx[t], b = idx[(t + 1) % m];
            if (a > b) { const int x = a; a = b; b = x; }
            int seen = -1;
            for (int e = 0; e < h->ne && seen < 0; ++e) if (h->e[e][0] == a && h->e[e][1] == b) seen = e;
            if (seen >= 0) h->ef[seen][1] = f;
            else if (h->ne < OR_HULL_MAXE) {
                h->e[h->ne][0] = a; h->e[h->ne][1] = b;
                h->ef[h->ne][0] = h->ef[h->ne][1] = f;
                ++h->ne;
            }
        }
    }
    return 1;
}

int or_hull_build(int np, const double* pts, or_hull_info* info)
{
    or_hull h;
    const int ok = or_hull_make(np, pts, &h);
    if (info) {
        info->nv = h.nv;
        info->nf = ok ? h.nf : 0;
        info->ne = ok ? h.ne : 0;
        for (int f = 0; f < info->nf; ++f) {
            info->n[f][0] = h.n[f][0]; info->n[f][1] = h.n[f][1]; info->n[f][2] = h.n[f][2];
            info->d[f] = h.d[f];
            info->fnv[f] = h.fnv[f];
            for (int k = 0; k < h.fnv[f]; ++k) info->fv[f][k] = h.fv[f][k];
        }
        for (int e = 0; e < info->ne; ++e) {
            info->e[e][0] = h.e[e][0]; info->e[e][1] = h.e[e][1];
            info->ef[e][0] = h.ef[e][0]; info->ef[e][1] = h.ef[e][1];
        }
    }
    return ok ? h.nf : 0;
}

/* the box as a hull: corners in the box slot order (bit 2: x, bit 1: y, bit 0: z) */
static void hull_box(const double* half, or_hull* h)
{
    double p[8][3];
    for (int c = 0; c < 8; ++c) {
        p[c][0] = (c & 4 ? 1.0 : -1.0) * half[0];
        p[c][1] = (c & 2 ? 1.0 : -1.0) * half[1];
        p[c][2] = (c & 1 ? 1.0 : -1.0) * half[2];
    }
    or_hull_make(8, &p[0][0], h);
}

/* closest points of segments p0 + s u, q0 + t v (s in [0, 1], t in [0, 1]) */
static void segment_closest(const double* p0, const double* p1, const double* q0, const double* q1, double* mid)
{
    double u[3], v[3], w[3];
    for (int k = 0; k < 3; ++k) { u[k] = p1[k] - p0[k]; v[k] = q1[k] - q0[k]; w[k] = p0[k] - q0[k]; }
    const double a = dot3(u, u), b = dot3(u, v), c = dot3(v, v), d = dot3(u, w), e = dot3(v, w);
    const double den = a * c - b * b;
    double s = den > 1e-18 * a * c ? (b * e - c * d) / den : 0.0;
    s = s < 0.0 ? 0.0 : (s > 1.0 ? 1.0 : s);
    double t = c > 0.0 ? (b * s + e) / c : 0.0;
    if (t < 0.0 || t > 1.0) {
        t = t < 0.0 ? 0.0 : 1.0;
        s = a > 0.0 ? (b * t - d) / a : 0.0;
        s = s < 0.0 ? 0.0 : (s > 1.0 ? 1.0 : s);
    }
    for (int k = 0; k < 3; ++k) mid[k] = 0.5 * ((p0[k] + s * u[k]) + (q0[k] + t * v[k]));
}

#define OR_HULL_CLIP 24   /* clipped polygon capacity (the scene kernel's kScClipMax) */

/* hull A vs hull B (shape frames at (cA, RA), (cB, RB)): the separating-axis
 * test over A's and B's face normals and every edge-pair direction (the
 * smallest overlap over those axes is the penetration depth of two convex
 * polytopes); the reference face is the face axis of least overlap (A's
 * unless B's is smaller by 5 % + 1e-5, as box_box prefers faces over edges),
 * the incident face the other hull's face most anti-parallel to it, clipped
 * against the reference face's side planes; an edge pair wins only below
 * 0.95 x the face overlap - 1e-5 (one point: the closest points' midpoint).
 * Normal from B into A, points on the incident surface, depths along it. */
static int hull_pair(const or_hull* A, const double* cA, const double* RA, const or_hull* B, const double* cB,
                     const double* RB, double n[3], double* pts, double* deps)
{
    double WA[OR_MESH_MAXP][3], WB[OR_MESH_MAXP][3], ca[3], cb[3];
    for (int i = 0; i < A->nv; ++i) mat_vec3(RA, A->v[i], cA, WA[i]);
    for (int i = 0; i < B->nv; ++i) mat_vec3(RB, B->v[i], cB, WB[i]);
    mat_vec3(RA, A->ctr, cA, ca);
    mat_vec3(RB, B->ctr, cB, cb);
    double pen[2] = {INFINITY, INFINITY};
    int face[2] = {-1, -1};
    for (int side = 0; side < 2; ++side) {
        const or_hull* H = side ? B : A;
        const double* R = side ? RB : RA;
        const double* c = side ? cB : cA;
        double (*Wo)[3] = side ? WA : WB;
        const int no = side ? A->nv : B->nv;
        for (int f = 0; f < H->nf; ++f) {
            double nw[3];
            rot3(R, H->n[f], nw);
            const double dw = H->d[f] + dot3(nw, c);
            double mn = INFINITY;
            for (int j = 0; j < no; ++j) {
                const double s = dot3(nw, Wo[j]);
                mn = s < mn ? s : mn;
            }
            const double ov = dw - mn;
            if (ov < 0.0) return 0;
            if (ov < pen[side]) { pen[side] = ov; face[side] = f; }
        }
    }
    double pen_e = INFINITY, eaxis[3] = {0, 0, 0};
    int ea = -1, eb = -1;
    for (int i = 0; i < A->ne; ++i)
        for (int j = 0; j < B->ne; ++j) {
            /* only edge pairs whose Gauss-map arcs cross (a face of the
             * Minkowski difference; Gregorius 2013): the others never hold
             * the least overlap */
            double a[3], b[3], c[3], d[3], bxa[3], dxc[3];
            rot3(RA, A->n[A->ef[i][0]], a);
            rot3(RA, A->n[A->ef[i][1]], b);
            rot3(RB, B->n[B->ef[j][0]], c);
            rot3(RB, B->n[B->ef[j][1]], d);
            for (int k = 0; k < 3; ++k) { c[k] = -c[k]; d[k] = -d[k]; }
            cross3(b, a, bxa);
            cross3(d, c, dxc);
            const double cba = dot3(c, bxa), dba = dot3(d, bxa), adc = dot3(a, dxc), bdc = dot3(b, dxc);
            if (!(cba * dba < 0.0 && adc * bdc < 0.0 && cba * bdc > 0.0)) continue;
            double da[3], db[3], u[3];
            for (int k = 0; k < 3; ++k) {
                da[k] = WA[A->e[i][1]][k] - WA[A->e[i][0]][k];
                db[k] = WB[B->e[j][1]][k] - WB[B->e[j][0]][k];
            }
            cross3(da, db, u);
            const double len = sqrt(dot3(u, u));
            if (len <= 1e-6 * sqrt(dot3(da, da) * dot3(db, db))) continue;   /* parallel edges */
            for (int k = 0; k < 3; ++k) u[k] /= len;
            const double dc[3] = {cb[0] - ca[0], cb[1] - ca[1], cb[2] - ca[2]};
            if (dot3(u, dc) < 0.0) for (int k = 0; k < 3; ++k) u[k] = -u[k];   /* A -> B */
            double amax = -INFINITY, bmin = INFINITY;
            for (int p = 0; p < A->nv; ++p) { const double s = dot3(u, WA[p]); amax = s > amax ? s : amax; }
            for (int p = 0; p < B->nv; ++p) { const double s = dot3(u, WB[p]); bmin = s < bmin ? s : bmin; }
            const double ov = amax - bmin;
            if (ov < 0.0) return 0;
            if (ov < pen_e) { pen_e = ov; ea = i; eb = j; memcpy(eaxis, u, sizeof u); }
        }
    const int refB = pen[1] < 0.95 * pen[0] - 1e-5;
    const double pen_f = refB ? pen[1] : pen[0];
    if (ea >= 0 && pen_e < 0.95 * pen_f - 1e-5) {
        for (int k = 0; k < 3; ++k) n[k] = -eaxis[k];
        segment_closest(WA[A->e[ea][0]], WA[A->e[ea][1]], WB[B->e[eb][0]], WB[B->e[eb][1]], pts);
        deps[0] = pen_e;
        return 1;
    }
    const or_hull* Rh = refB ? B : A;
    const or_hull* Ih = refB ? A : B;
    const double* Rr = refB ? RB : RA;
    const double* Ri = refB ? RA : RB;
    double (*Wr)[3] = refB ? WB : WA;
    double (*Wi)[3] = refB ? WA : WB;
    const int fr = face[refB ? 1 : 0];
    double nr[3];
    rot3(Rr, Rh->n[fr], nr);                           /* reference normal, pointing to the incident hull */
    const double dr = Rh->d[fr] + dot3(nr, refB ? cB : cA);
    int fi = 0;
    double best = INFINITY;
    for (int f = 0; f < Ih->nf; ++f) {
        double nw[3];
        rot3(Ri, Ih->n[f], nw);
        const double s = dot3(nw, nr);
        if (s < best) { best = s; fi = f; }
    }
    double buf[2][OR_HULL_CLIP][3];
    int cnt = Ih->fnv[fi], cur = 0;
    for (int k = 0; k < cnt; ++k) memcpy(buf[0][k], Wi[Ih->fv[fi][k]], sizeof buf[0][k]);
    for (int k = 0; k < Rh->fnv[fr] && cnt > 0; ++k) {
        const double* r0 = Wr[Rh->fv[fr][k]];
        const double* r1 = Wr[Rh->fv[fr][(k + 1) % Rh->fnv[fr]]];
        double e[3] = {r1[0] - r0[0], r1[1] - r0[1], r1[2] - r0[2]}, sn[3];
        cross3(e, nr, sn);                              /* outward side-plane normal */
        int m = 0;
        for (int i = 0; i < cnt; ++i) {
            const double* P = buf[cur][i];
            const double* Q = buf[cur][(i + 1) % cnt];
            const double dp = dot3(sn, P) - dot3(sn, r0), dq = dot3(sn, Q) - dot3(sn, r0);
            if (dp <= 0.0 && m < OR_HULL_CLIP) memcpy(buf[cur ^ 1][m++], P, sizeof buf[0][0]);
            if (((dp < 0.0 && dq > 0.0) || (dp > 0.0 && dq < 0.0)) && m < OR_HULL_CLIP) {
                const double t = dp / (dp - dq);
                for (int q = 0; q < 3; ++q) buf[cur ^ 1][m][q] = P[q] + t * (Q[q] - P[q]);
                ++m;
            }
        }
        cnt = m;
        cur ^= 1;
    }
    double P8[OR_HULL_CLIP][3], D8[OR_HULL_CLIP];
    int np = 0;
    for (int i = 0; i < cnt; ++i) {
        const double dep = dr - dot3(nr, buf[cur][i]);
        if (dep > 0.0) { memcpy(P8[np], buf[cur][i], sizeof P8[np]); D8[np] = dep; ++np; }
    }
    np = reduce_points(np, P8, D8);
    for (int k = 0; k < 3; ++k) n[k] = refB ? nr[k] : -nr[k];
    for (int i = 0; i < np; ++i) {
        memcpy(pts + 3 * i, P8[i], 3 * sizeof(double));
        deps[i] = D8[i];
    }
    return np;
}

/* A mesh whose support points are exactly its bounding box's 8 corners is
 * that box (it collides through box_box, bit for bit like the box). */
static int mesh_is_box(int type, const double* size, int npts, const double* pts)
{
    if (type != 3 || npts != 8) return 0;
    int corners = 0;
    for (int i = 0; i < 8; ++i) {
        int ok = 1;
        for (int k = 0; k < 3; ++k) ok = ok && fabs(fabs(pts[3 * i + k]) - size[k]) <= 1e-12 * (1.0 + size[k]);
        corners |= ok << ((pts[3 * i] > 0) * 4 + (pts[3 * i + 1] > 0) * 2 + (pts[3 * i + 2] > 0));
    }
    return corners == 0xff;
}

/* a mesh shape (type 3) against a box or another mesh: the hull narrow
 * phase; npts / pts: the mesh shapes' support points (shape frame) */
int or_collide_hull(int type_a, const double* size_a, int npts_a, const double* pts_a, const double* c_a,
                    const double* R_a, int type_b, const double* size_b, int npts_b, const double* pts_b,
                    const double* c_b, const double* R_b, double normal[3], double* points, double* depths)
{
    static _Thread_local or_hull ha, hb;
    if (type_a == 3) { if (!or_hull_make(npts_a, pts_a, &ha)) hull_box(size_a, &ha); } else hull_box(size_a, &ha);
    if (type_b == 3) { if (!or_hull_make(npts_b, pts_b, &hb)) hull_box(size_b, &hb); } else hull_box(size_b, &hb);
    return hull_pair(&ha, c_a, R_a, &hb, c_b, R_b, normal, points, depths);
}

int or_collide(int type_a, const double* size_a, const double* c_a, const double* R_a, int type_b,
               const double* size_b, const double* c_b, const double* R_b, double normal[3], double* points,
               double* depths)
{
    if ((type_a == 2 && type_b == 1) || (type_a == 1 && type_b == 2)) {
        double nbs[3];
        if (type_a == 2) {   /* cylinder A, sphere B: n from B into A */
            if (!cylinder_sphere(size_a, c_a, R_a, size_b[0], c_b, nbs, points, depths)) return 0;
            for (int k = 0; k < 3; ++k) normal[k] = -nbs[k];
            return 1;
        }
        if (!cylinder_sphere(size_b, c_b, R_b, size_a[0], c_a, nbs, points, depths)) return 0;
        memcpy(normal, nbs, sizeof nbs);
        return 1;
    }
    if (type_a == 2 || type_b == 2)   /* cylinder-box, cylinder-cylinder */
        return cylinder_pair(type_a, size_a, c_a, R_a, type_b, size_b, c_b, R_b, normal, points, depths);
    if (type_a == 0 && type_b == 0) return box_box(size_a, c_a, R_a, size_b, c_b, R_b, normal, points, depths);
    if (type_a == 1 && type_b == 1) {
        double d[3] = {c_a[0] - c_b[0], c_a[1] - c_b[1], c_a[2] - c_b[2]};
        const double dist = sqrt(dot3(d, d));
        const double pen = size_a[0] + size_b[0] - dist;
        if (pen < 0.0 || dist < 1e-12) return 0;
        for (int k = 0; k < 3; ++k) normal[k] = d[k] / dist;
        for (int k = 0; k < 3; ++k) points[k] = c_b[k] + normal[k] * (size_b[0] - 0.5 * pen);
        depths[0] = pen;
        return 1;
    }
    double nbs[3];
    if (type_a == 0) {   /* box A, sphere B: n from B into A = -(box -> sphere) */
        if (!box_sphere(size_a, c_a, R_a, size_b[0], c_b, nbs, points, depths)) return 0;
        for (int k = 0; k < 3; ++k) normal[k] = -nbs[k];
        return 1;
    }
    if (!box_sphere(size_b, c_b, R_b, size_a[0], c_a, nbs, points, depths)) return 0;
    memcpy(normal, nbs, sizeof nbs);
    return 1;
}

/* dense solve with pivoting for the scene (n <= OR_SC_MAXNV) */
static void scene_solve(int n, const double* A_in, const double* b, double* x)
{
    static _Thread_local double A[OR_SC_MAXNV * OR_SC_MAXNV];
    double y[OR_SC_MAXNV];
    memcpy(A, A_in, (size_t)n * n * sizeof(double));
    memcpy(y, b, (size_t)n * sizeof(double));
    (void)lcp_gauss(n, A, y, x);
}

/* world pose of link `b` (-1 = base) of model m */
static void scene_link_pose(const or_float_state* s, const or_fkin* k, int b, const double** R, const double** p)
{
    *R = b < 0 ? s->R : k->Rw[b];
    *p = b < 0 ? s->p : k->pw[b];
}

int or_scene_step(const or_scene_model* sm, double dt, or_scene_state* st, const int32_t* mode,
                  const double* cmd, const double* wrench, int pgs_iters, double* c_out, int32_t* c_who)
{
    const int K = sm->n_models;
    static _Thread_local or_fkin kin[OR_SC_MAXM];
    int off[OR_SC_MAXM], nbase[OR_SC_MAXM];
    g_cap_n = 0;  /* a step without rows leaves no capture behind */
    int NV = 0;
    for (int m = 0; m < K; ++m) {
        off[m] = NV;
        nbase[m] = sm->floating[m] ? 6 : 0;
        NV += nbase[m] + sm->model[m].tree.n;
        float_kin(&sm->model[m], &st->s[m], &kin[m]);
    }
    /* block-diagonal M, h; rhs with damping, commands and wrenches */
    static _Thread_local double M[OR_SC_MAXNV * OR_SC_MAXNV], Mi[OR_SC_MAXNV * OR_SC_MAXNV];
    double rhs[OR_SC_MAXNV], acc[OR_SC_MAXNV], nu[OR_SC_MAXNV];
    for (int e = 0; e < NV * NV; ++e) M[e] = 0.0;
    for (int m = 0; m < K; ++m) {
        const or_float_model* fm = &sm->model[m];
        const or_model* t = &fm->tree;
        const int n = t->n, nvm = 6 + n, nb = nbase[m], o = off[m];
        static _Thread_local double Mm[(6 + OR_MAXB) * (6 + OR_MAXB)];
        double hm[6 + OR_MAXB];
        or_float_model tmp = *fm;
        for (int r = 0; r < 3; ++r) tmp.gravity[r] = sm->gravity[r];
        or_float_state s0 = st->s[m];
        if (!sm->floating[m]) memset(s0.V, 0, sizeof s0.V);
        or_float_dynamics(&tmp, &s0, Mm, hm);
        for (int r = 6 - nb; r < nvm; ++r)
            for (int c = 6 - nb; c < nvm; ++c) M[(o + r - 6 + nb) * NV + o + c - 6 + nb] = Mm[r * nvm + c];
        for (int r = 6 - nb; r < nvm; ++r) rhs[o + r - 6 + nb] = -hm[r];
        for (int e = 0; e < nb; ++e) nu[o + e] = s0.V[e];
        for (int i = 0; i < n; ++i) {
            const int j = o + nb + i;
            double tau = 0.0;
            if (mode[m * OR_MAXB + i] == OR_FORCE) {
                tau = cmd[m * OR_MAXB + i];
                if (tau < -t->effort[i]) tau = -t->effort[i];
                if (tau > t->effort[i]) tau = t->effort[i];
            }
            rhs[j] += tau - t->damping[i] * s0.qd[i];
            nu[j] = s0.qd[i];
        }
        if (wrench) {
            for (int b = -1; b < n; ++b) {
                const double* wr = wrench + ((size_t)m * (1 + OR_MAXB) + (size_t)(b + 1)) * 6;
                if (wr[0] == 0.0 && wr[1] == 0.0 && wr[2] == 0.0 && wr[3] == 0.0 && wr[4] == 0.0 && wr[5] == 0.0)
                    continue;
                const double *Rl, *pl;
                scene_link_pose(&s0, &kin[m], b, &Rl, &pl);
                /* body-frame spatial force [R^T torque; R^T force] at the link origin */
                double f[6], J[6 + OR_MAXB];
                for (int r = 0; r < 3; ++r) {
                    f[r] = Rl[r] * wr[3] + Rl[3 + r] * wr[4] + Rl[6 + r] * wr[5];
                    f[3 + r] = Rl[r] * wr[0] + Rl[3 + r] * wr[1] + Rl[6 + r] * wr[2];
                }
                if (b < 0) {
                    for (int e = 0; e < nvm; ++e) J[e] = 0.0;
                    for (int e = 0; e < 6; ++e) J[e] = f[e];
                } else {
                    float_row(fm, &kin[m], b, f, J);
                }
                for (int r = 6 - nb; r < nvm; ++r) rhs[o + r - 6 + nb] += J[r];
            }
        }
    }
    memcpy(Mi, M, (size_t)NV * NV * sizeof(double));
    for (int m = 0; m < K; ++m)
        for (int i = 0; i < sm->model[m].tree.n; ++i) {
            const int j = off[m] + nbase[m] + i;
            Mi[j * NV + j] += dt * sm->model[m].tree.damping[i];
        }
    scene_solve(NV, Mi, rhs, acc);
    for (int e = 0; e < NV; ++e) nu[e] += dt * acc[e];

    /* ---- contacts ---- */
    int nc = 0;
    double cp[OR_SC_MAXC][3], cn[OR_SC_MAXC][3], cd[OR_SC_MAXC];
    int who[OR_SC_MAXC][4];
    if (sm->ground) {
        for (int m = 0; m < K; ++m) {
            const or_float_model* fm = &sm->model[m];
            for (int sh = 0; sh < fm->n_shapes; ++sh) {
                const int bi = fm->shape_body[sh];
                if (bi < 0 && !sm->floating[m]) continue;   /* a welded base link does not move */
                const double *Rb, *pb;
                scene_link_pose(&st->s[m], &kin[m], bi, &Rb, &pb);
                const double* hh = fm->shape_size[sh];
                const double* SR = fm->shape_R[sh];
                const double* sp = fm->shape_p[sh];
                const int corners = (fm->shape_type[sh] == 1) ? 1 : (fm->shape_type[sh] == 3) ? fm->shape_npts[sh] : 8;
                double RS[9];
                rot_mul(Rb, SR, RS);
                for (int corner = 0; corner < corners; ++corner) {
                    double l[3], b3[3], x[3];
                    if (fm->shape_type[sh] == 3)   /* mesh: its support points */
                        memcpy(l, fm->shape_pts[sh][corner], sizeof l);
                    else
                        or_slot_point(fm->shape_type[sh], hh, RS, corner, l);
                    for (int r = 0; r < 3; ++r) b3[r] = sp[r] + SR[r * 3] * l[0] + SR[r * 3 + 1] * l[1] + SR[r * 3 + 2] * l[2];
                    for (int r = 0; r < 3; ++r) x[r] = pb[r] + Rb[r * 3] * b3[0] + Rb[r * 3 + 1] * b3[1] + Rb[r * 3 + 2] * b3[2];
                    double dep = -x[2];
                    if (fm->shape_type[sh] == 1) {
                        dep = hh[0] - x[2];
                        x[2] -= hh[0];
                    }
                    if (dep > 0.0 && nc < OR_SC_MAXC) {
                        memcpy(cp[nc], x, sizeof x);
                        cn[nc][0] = 0.0; cn[nc][1] = 0.0; cn[nc][2] = 1.0;
                        cd[nc] = dep;
                        who[nc][0] = m; who[nc][1] = bi; who[nc][2] = -1; who[nc][3] = -1;
                        ++nc;
                    }
                }
            }
        }
    }
    for (int ma = 0; ma < K; ++ma)
        for (int sa = 0; sa < sm->model[ma].n_shapes; ++sa)
            for (int mb = ma + 1; mb < K; ++mb)
                for (int sb = 0; sb < sm->model[mb].n_shapes; ++sb) {
                    double cA[3], RA[9], cB[3], RB[9];
                    const or_float_model* A = &sm->model[ma];
                    const or_float_model* B = &sm->model[mb];
                    const int ba = A->shape_body[sa], bb = B->shape_body[sb];
                    if (ba < 0 && !sm->floating[ma] && bb < 0 && !sm->floating[mb]) continue;  /* both welded */
                    for (int side = 0; side < 2; ++side) {
                        const or_float_model* F = side ? B : A;
                        const int sh = side ? sb : sa;
                        const double *Rl, *pl;
                        scene_link_pose(&st->s[side ? mb : ma], &kin[side ? mb : ma], side ? bb : ba, &Rl, &pl);
                        double* c = side ? cB : cA;
                        double* R = side ? RB : RA;
                        for (int r = 0; r < 3; ++r) {
                            c[r] = pl[r] + Rl[r * 3] * F->shape_p[sh][0] + Rl[r * 3 + 1] * F->shape_p[sh][1] +
                                   Rl[r * 3 + 2] * F->shape_p[sh][2];
                            for (int q = 0; q < 3; ++q)
                                R[r * 3 + q] = Rl[r * 3] * F->shape_R[sh][q] + Rl[r * 3 + 1] * F->shape_R[sh][3 + q] +
                                               Rl[r * 3 + 2] * F->shape_R[sh][6 + q];
                        }
                    }
                    double nrm[3], pts[12], deps[4];
                    const int ta0 = A->shape_type[sa], tb0 = B->shape_type[sb];
                    int np;
                    const int ta1 = mesh_is_box(ta0, A->shape_size[sa], A->shape_npts[sa], &A->shape_pts[sa][0][0])
                                        ? 0 : ta0;
                    const int tb1 = mesh_is_box(tb0, B->shape_size[sb], B->shape_npts[sb], &B->shape_pts[sb][0][0])
                                        ? 0 : tb0;
                    if ((ta1 == 3 && (tb1 == 0 || tb1 == 3)) || (tb1 == 3 && ta1 == 0)) {
                        /* a mesh against a box or a mesh: the hull narrow phase */
                        np = or_collide_hull(ta1, A->shape_size[sa], A->shape_npts[sa], &A->shape_pts[sa][0][0], cA,
                                             RA, tb1, B->shape_size[sb], B->shape_npts[sb], &B->shape_pts[sb][0][0],
                                             cB, RB, nrm, pts, deps);
                    } else {
                        /* a box-shaped mesh is its box; a mesh against a sphere or a
                         * cylinder: its bounding box */
                        const int ta = ta1 == 3 ? 0 : ta1, tb = tb1 == 3 ? 0 : tb1;
                        np = or_collide(ta, A->shape_size[sa], cA, RA, tb, B->shape_size[sb], cB, RB, nrm, pts, deps);
                    }
                    for (int i = 0; i < np && nc < OR_SC_MAXC; ++i) {
                        memcpy(cp[nc], pts + 3 * i, sizeof cp[nc]);
                        memcpy(cn[nc], nrm, sizeof nrm);
                        cd[nc] = deps[i];
                        who[nc][0] = ma; who[nc][1] = ba; who[nc][2] = mb; who[nc][3] = bb;
                        ++nc;
                    }
                }

    /* ---- rows: contacts (normal, t1, t2), then joint rows model by model ---- */
    enum { K_NORMAL, K_FRIC, K_BOX };
    const int maxr = 3 * OR_SC_MAXC + 3 * OR_MAXB;
    static _Thread_local double J[3 * OR_SC_MAXC + 3 * OR_MAXB][OR_SC_MAXNV];
    static _Thread_local double MJ[3 * OR_SC_MAXC + 3 * OR_MAXB][OR_SC_MAXNV];
    static _Thread_local double A[(3 * OR_SC_MAXC + 3 * OR_MAXB) * (3 * OR_SC_MAXC + 3 * OR_MAXB)];
    static _Thread_local double bb[3 * OR_SC_MAXC + 3 * OR_MAXB], lo[3 * OR_SC_MAXC + 3 * OR_MAXB],
        hi[3 * OR_SC_MAXC + 3 * OR_MAXB], cfm[3 * OR_SC_MAXC + 3 * OR_MAXB], x[3 * OR_SC_MAXC + 3 * OR_MAXB];
    static _Thread_local int kind[3 * OR_SC_MAXC + 3 * OR_MAXB];
    (void)maxr;
    int nr = 0;
    double tb1[OR_SC_MAXC][3], tb2[OR_SC_MAXC][3];
    for (int c = 0; c < nc; ++c) {
        plane_space(cn[c], tb1[c], tb2[c]);
        for (int d = 0; d < 3; ++d) {
            const double* dw = d == 0 ? cn[c] : (d == 1 ? tb1[c] : tb2[c]);
            for (int e = 0; e < NV; ++e) J[nr][e] = 0.0;
            for (int side = 0; side < 2; ++side) {
                const int m = who[c][2 * side], b = who[c][2 * side + 1];
                if (m < 0) continue;
                const double sg = side ? -1.0 : 1.0;
                const or_float_model* fm = &sm->model[m];
                const double *Rl, *pl;
                scene_link_pose(&st->s[m], &kin[m], b, &Rl, &pl);
                const double rel[3] = {cp[c][0] - pl[0], cp[c][1] - pl[1], cp[c][2] - pl[2]};
                double f[6], bp[3], Jm[6 + OR_MAXB];
                for (int r = 0; r < 3; ++r) {
                    f[3 + r] = Rl[r] * dw[0] + Rl[3 + r] * dw[1] + Rl[6 + r] * dw[2];
                    bp[r] = Rl[r] * rel[0] + Rl[3 + r] * rel[1] + Rl[6 + r] * rel[2];
                }
                cross3(bp, f + 3, f);
                const int nvm = 6 + fm->tree.n;
                if (b < 0) {
                    for (int e = 0; e < nvm; ++e) Jm[e] = 0.0;
                    for (int e = 0; e < 6; ++e) Jm[e] = f[e];
                } else {
                    float_row(fm, &kin[m], b, f, Jm);
                }
                const int nb = nbase[m];
                for (int r = 6 - nb; r < nvm; ++r) J[nr][off[m] + r - 6 + nb] += sg * Jm[r];
            }
            double vrel = 0.0;
            for (int e = 0; e < NV; ++e) vrel += J[nr][e] * nu[e];
            double bounce = 0.0;
            if (d == 0) {
                bounce = OR_C_ERP * cd[c] / dt;
                if (bounce > OR_C_MAX_ERV) bounce = OR_C_MAX_ERV;
            }
            bb[nr] = -vrel + bounce;
            kind[nr] = d == 0 ? K_NORMAL : K_FRIC;
            lo[nr] = 0.0;
            hi[nr] = INFINITY;
            cfm[nr] = OR_C_CFM;
            ++nr;
        }
    }
    for (int m = 0; m < K; ++m) {
        const or_model* t = &sm->model[m].tree;
        const or_float_state* s = &st->s[m];
        for (int i = 0; i < t->n; ++i) {
            const int col = off[m] + nbase[m] + i;
            const double qdi = nu[col];
            int rows_i[3], nri = 0;
            if (t->limited[i]) {
                double viol = s->q[i] - t->lower[i];
                int active = 0;
                if (viol <= 0.0) { lo[nr] = 0.0; hi[nr] = INFINITY; active = 1; }
                else {
                    viol = s->q[i] - t->upper[i];
                    if (viol >= 0.0) { lo[nr] = -INFINITY; hi[nr] = 0.0; active = 1; }
                }
                if (active) {
                    double bounce = -viol * OR_ERP / dt;
                    if (bounce > OR_MAX_ERV) bounce = OR_MAX_ERV;
                    if (bounce < -OR_MAX_ERV) bounce = -OR_MAX_ERV;
                    bb[nr] = -qdi + bounce;
                    rows_i[nri++] = nr++;
                }
            }
            if (mode[m * OR_MAXB + i] == OR_SERVO) {
                double vc = cmd[m * OR_MAXB + i];
                if (vc < -t->vel_limit[i]) vc = -t->vel_limit[i];
                if (vc > t->vel_limit[i]) vc = t->vel_limit[i];
                if (vc - qdi != 0.0) {
                    bb[nr] = vc - qdi;
                    lo[nr] = -t->effort[i] * dt;
                    hi[nr] = t->effort[i] * dt;
                    rows_i[nri++] = nr++;
                }
            }
            if (t->friction[i] != 0.0 && qdi != 0.0) {
                bb[nr] = -qdi;
                hi[nr] = t->friction[i] * dt;
                lo[nr] = -hi[nr];
                rows_i[nri++] = nr++;
            }
            for (int r = 0; r < nri; ++r) {
                const int row = rows_i[r];
                for (int e = 0; e < NV; ++e) J[row][e] = 0.0;
                J[row][col] = 1.0;
                kind[row] = K_BOX;
                cfm[row] = OR_CFM;
            }
        }
    }
    if (nr > 0) {
        for (int r = 0; r < nr; ++r) scene_solve(NV, M, J[r], MJ[r]);
        for (int r = 0; r < nr; ++r) {
            for (int c = 0; c < nr; ++c) {
                double a = 0.0;
                for (int e = 0; e < NV; ++e) a += J[r][e] * MJ[c][e];
                A[r * nr + c] = a;
            }
            A[r * nr + r] *= 1.0 + cfm[r];
            x[r] = 0.0;
        }
        if (nr <= OR_CAP_MAXN) {
            g_cap_n = nr;
            g_cap_mu = sm->mu;
            for (int r = 0; r < nr; ++r) {
                for (int c = 0; c < nr; ++c) g_cap_A[r * nr + c] = A[r * nr + c];
                g_cap_b[r] = bb[r];
                g_cap_wid[r] = -1;
                g_cap_bscale[r] = fabs(bb[r]);
                g_cap_x1[r] = 0.0;
                g_cap_kind[r] = kind[r];
                g_cap_lo[r] = kind[r] == K_BOX ? lo[r] : (kind[r] == K_NORMAL ? 0.0 : -INFINITY);
                g_cap_hi[r] = kind[r] == K_BOX ? hi[r] : INFINITY;
            }
        }
        g_pgs_sweeps = 0;
        for (int it = 0; it < pgs_budget(pgs_iters); ++it) {
            for (int r = 0; r < nr; ++r) {
                double acc_r = bb[r];
                for (int c = 0; c < nr; ++c) acc_r -= A[r * nr + c] * x[c];
                double v = x[r] + acc_r / A[r * nr + r];
                double l = lo[r], u = hi[r];
                if (kind[r] == K_FRIC) {
                    u = sm->mu * x[r - (r % 3)];
                    l = -u;
                }
                if (v < l) v = l;
                if (v > u) v = u;
                x[r] = v;
            }
            pgs_count(it);
        }
        if (pgs_iters < 0) {
            static _Thread_local int findex[3 * OR_SC_MAXC + 3 * OR_MAXB];
            for (int r = 0; r < nr; ++r) findex[r] = (kind[r] == K_FRIC) ? r - (r % 3) : -1;
            lcp_dantzig(nr, A, nr, bb, lo, hi, findex, sm->mu, x);
            if (nr <= OR_CAP_MAXN)
                for (int r = 0; r < nr; ++r) g_cap_x1[r] = g_last_x1[r];
        }
        if (nr <= OR_CAP_MAXN)
            for (int r = 0; r < nr; ++r) g_cap_x[r] = x[r];
        for (int r = 0; r < nr; ++r)
            for (int e = 0; e < NV; ++e) nu[e] += MJ[r][e] * x[r];
    }

    /* ---- integratePositions ---- */
    for (int m = 0; m < K; ++m) {
        or_float_state* s = &st->s[m];
        const int o = off[m], nb = nbase[m];
        for (int i = 0; i < sm->model[m].tree.n; ++i) s->qd[i] = nu[o + nb + i];
        integrate_joint_positions(&sm->model[m].tree, s->q, s->qd, dt);
        if (!nb) continue;
        double phi[3] = {dt * nu[o], dt * nu[o + 1], dt * nu[o + 2]};
        double u[3] = {dt * nu[o + 3], dt * nu[o + 4], dt * nu[o + 5]};
        double dR[9], dp[3], Rn[9];
        se3_exp(phi, u, dR, dp);
        for (int r = 0; r < 3; ++r) {
            s->p[r] += s->R[r * 3] * dp[0] + s->R[r * 3 + 1] * dp[1] + s->R[r * 3 + 2] * dp[2];
            for (int q = 0; q < 3; ++q)
                Rn[r * 3 + q] = s->R[r * 3] * dR[q] + s->R[r * 3 + 1] * dR[3 + q] + s->R[r * 3 + 2] * dR[6 + q];
        }
        memcpy(s->R, Rn, sizeof Rn);
        for (int e = 0; e < 6; ++e) s->V[e] = nu[o + e];
    }
    for (int c = 0; c < nc; ++c) {
        if (c_out) {
            double* o = c_out + 10 * c;
            for (int r = 0; r < 3; ++r) {
                o[r] = cp[c][r];
                o[3 + r] = cn[c][r];
                o[6 + r] = (cn[c][r] * x[3 * c] + tb1[c][r] * x[3 * c + 1] + tb2[c][r] * x[3 * c + 2]) / dt;
            }
            o[9] = cd[c];
        }
        if (c_who) memcpy(c_who + 4 * c, who[c], sizeof who[c]);
    }
    return nc;
}

/* ------------------------------------------------------------------ */
/* CPU-baseline rollouts (bench.py's cpu_baseline of BASELINE configs 4 */
/* and 5): T engine steps under the JointController PID hold, in C so   */
/* the timing is the oracle's physics, not Python.  Error = q - target  */
/* (JointController.cpp:308), the PID every step (period = dt).         */
/* ------------------------------------------------------------------ */

/* W fixed-base worlds [W][n]: targets q0 + amp sin(2 pi freq t). */
void or_pid_rollout(const or_model* m, double dt, int W, int T, double* q, double* qd, const double* q0,
                    const double* amp, double freq, const or_pid_gains* g, or_pid_state* st, int pgs_iters)
{
    const int n = m->n;
    int32_t mode[OR_MAXB];
    double tau[OR_MAXB], qdd[OR_MAXB], frc[OR_MAXB];
    for (int i = 0; i < n; ++i) mode[i] = OR_FORCE;
    for (int t = 0; t < T; ++t) {
        const double s = sin(2.0 * OR_PI * freq * (t + 1) * dt);
        for (int w = 0; w < W; ++w) {
            double* qw = q + (size_t)w * n;
            double* qdw = qd + (size_t)w * n;
            for (int i = 0; i < n; ++i)
                tau[i] = or_pid_update(&g[i], &st[(size_t)w * n + i], qw[i] - (q0[(size_t)w * n + i] + amp[i] * s), dt);
            or_step(m, dt, qw, qdw, mode, tau, pgs_iters, qdd, frc);
        }
    }
}

/* One floating-base world, targets fixed (the humanoid's PID hold). */
void or_float_pid_rollout(const or_float_model* m, double dt, int T, or_float_state* s, const double* target,
                          const or_pid_gains* g, or_pid_state* st, int pgs_iters)
{
    const int n = m->tree.n;
    int32_t mode[OR_MAXB];
    double tau[OR_MAXB];
    static _Thread_local double cp[3 * OR_MAXFC], cf[3 * OR_MAXFC], cd[OR_MAXFC];
    static _Thread_local int32_t cb[OR_MAXFC];
    for (int i = 0; i < n; ++i) mode[i] = OR_FORCE;
    for (int t = 0; t < T; ++t) {
        for (int i = 0; i < n; ++i) tau[i] = or_pid_update(&g[i], &st[i], s->q[i] - target[i], dt);
        or_float_step(m, dt, s, mode, tau, pgs_iters, cp, cf, cd, cb);
    }
}

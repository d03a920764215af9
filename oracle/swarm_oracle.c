/*
 * swarm_oracle.c — CPU restatement of the SwarmACB e-puck env step.
 *
 * TEST INFRASTRUCTURE ONLY (see swarm_oracle.h). Written to follow the
 * reference's tensor expressions op-for-op in fp32 so that teacher-forced
 * steps agree with the golden vectors within 1e-5. Reference paths:
 *   ES = source/.../tasks/direct/epuck/epuck_sensors.py
 *   BM = source/.../tasks/direct/epuck/behavior_modules.py
 *   DG = source/.../missions/directional_gate/directional_gate_env.py (+ _cfg DGC)
 *   HM/XO/FO/SH = homing / xor_aggregation / foraging / sheltering envs
 *   MC = scripts/manual_control.py (StandaloneDGTEnv, the north-star oracle)
 * Every scalar constant is computed in double (as Python does) and rounded to
 * float where torch would cast a Python scalar into a float32 tensor op.
 */
#include "swarm_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define PI_D 3.14159265358979323846

/* ------------------------------------------------------------------------ */
/*  Private generator: MT19937 (torch CPU generator stream; used only when a */
/*  draw is not replayed, i.e. for the CPU-baseline timing).                */
/* ------------------------------------------------------------------------ */
static uint32_t mt_[624];
static int mti_ = 625;

void or_seed(uint64_t seed) {
    mt_[0] = (uint32_t)seed;
    for (mti_ = 1; mti_ < 624; mti_++)
        mt_[mti_] = 1812433253u * (mt_[mti_ - 1] ^ (mt_[mti_ - 1] >> 30)) + (uint32_t)mti_;
}

static uint32_t mt_next(void) {
    if (mti_ >= 624) {
        if (mti_ == 625) or_seed(5489u);
        for (int k = 0; k < 624; k++) {
            uint32_t y = (mt_[k] & 0x80000000u) | (mt_[(k + 1) % 624] & 0x7fffffffu);
            mt_[k] = mt_[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        mti_ = 0;
    }
    uint32_t y = mt_[mti_++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}
static float mt_uniform(void) { return (float)(mt_next() & 0xFFFFFFu) * (1.0f / 16777216.0f); }
static int32_t mt_randint(int lo, int hi) { return lo + (int32_t)(mt_next() % (uint32_t)(hi - lo)); }

/* ------------------------------------------------------------------------ */
/*  Geometry / constants                                                    */
/* ------------------------------------------------------------------------ */
#define MAXSEG 16
typedef struct {
    int nseg;                 /* arena (12) + internal walls */
    float seg[MAXSEG][4];     /* torch.tensor(segments, float32) (ES:205) */
    int nint;                 /* internal wall segments (DG gate / SH shelter) */
    double iseg[4][4];        /* the same internal segments in double (DG:916) */
    float face_n[12][2], face_p[12][2];   /* DG:849-872 */
    float mcf_n[12][2], mcf_p[12][2];     /* MC:536-544 (with its own mid-angle) */
    int has_light;
    float light[2];
    /* sensor geometry (ES:28-41, 75-79) */
    float cos_a[8], sin_a[8];
    float rab_cos[4], rab_sin[4];
    /* mission geometry (double, as in the cfg) */
    double ni, corr_south, gate_south, corr_hw, gate_hw, side_wall_len;
    double shelter[4];        /* left, right, bottom, top */
    double nest_top;
} geom;

static void build_geom(const or_cfg* c, geom* g) {
    memset(g, 0, sizeof(*g));
    const int n = 12;
    const double R = sqrt(2 * 4.91 / (n * sin(2 * PI_D / n)));        /* DGC:34-36, MC:113 */
    double vx[12], vy[12];
    for (int i = 0; i < n; i++) {                                       /* DG:615-628 */
        double a = 2 * PI_D * i / n + PI_D / n;
        vx[i] = R * cos(a);
        vy[i] = R * sin(a);
    }
    for (int i = 0; i < n; i++) {
        double ax = vx[i], ay = vy[i], bx = vx[(i + 1) % n], by = vy[(i + 1) % n];
        g->seg[i][0] = (float)ax; g->seg[i][1] = (float)ay;
        g->seg[i][2] = (float)bx; g->seg[i][3] = (float)by;
        double mx = 0.5 * (ax + bx), my = 0.5 * (ay + by);               /* DG:858-868 */
        double nrm = sqrt(mx * mx + my * my) + 1e-12;
        g->face_n[i][0] = (float)(-mx / nrm); g->face_n[i][1] = (float)(-my / nrm);
        g->face_p[i][0] = (float)mx; g->face_p[i][1] = (float)my;
    }
    g->ni = R * cos(PI_D / n);                                          /* DG:649-650 */
    for (int i = 0; i < n; i++) {                                       /* MC:536-544 */
        double a1 = 2 * PI_D * i / n + PI_D / n;
        double a2 = 2 * PI_D * ((i + 1) % n) / n + PI_D / n;
        double mid = (a1 + a2) / 2.0;
        g->mcf_n[i][0] = (float)(-cos(mid)); g->mcf_n[i][1] = (float)(-sin(mid));
        g->mcf_p[i][0] = (float)(g->ni * cos(mid)); g->mcf_p[i][1] = (float)(g->ni * sin(mid));
    }
    g->nseg = n;
    g->corr_south = g->ni - 1.06;                                       /* DG:652-656 */
    g->gate_south = g->corr_south - 0.33;
    g->corr_hw = 0.50 / 2.0;
    g->gate_hw = 0.45 / 2.0;
    g->side_wall_len = 0.50;
    g->shelter[0] = 0.0 - 0.50 / 2; g->shelter[1] = 0.0 + 0.50 / 2;    /* SH:24-27 */
    g->shelter[2] = 0.0 - 0.30 / 2; g->shelter[3] = 0.0 + 0.30 / 2;
    if (c->profile == OR_STANDALONE) {
        /* MC:322-329 goes through float32 tensors then .item() */
        float half0 = 0.50f / 2.0f, half1 = 0.30f / 2.0f;
        g->shelter[0] = (double)(0.0f - half0); g->shelter[1] = (double)(0.0f + half0);
        g->shelter[2] = (double)(0.0f - half1); g->shelter[3] = (double)(0.0f + half1);
    }
    g->nest_top = (c->profile == OR_STANDALONE) ? -0.63 : -0.58;       /* MC:162, FOC:28 */

    /* internal walls: DG:630-645 (2 side walls) / SH:29-35 (3 shelter walls) */
    g->nint = 0;
    if (c->mission == OR_DGT) {
        double hw = g->corr_hw, gs = g->gate_south, wl = g->side_wall_len;
        double s[2][4] = {{-hw, gs, -hw, gs + wl}, {hw, gs, hw, gs + wl}};
        for (int k = 0; k < 2; k++) memcpy(g->iseg[k], s[k], sizeof(s[k]));
        g->nint = 2;
    } else if (c->mission == OR_SHELTERING) {
        double l = g->shelter[0], r = g->shelter[1], b = g->shelter[2], t = g->shelter[3];
        double s[3][4] = {{l, b, l, t}, {r, b, r, t}, {l, t, r, t}};
        for (int k = 0; k < 3; k++) memcpy(g->iseg[k], s[k], sizeof(s[k]));
        g->nint = 3;
    }
    for (int k = 0; k < g->nint; k++) {
        for (int q = 0; q < 4; q++) g->seg[n + k][q] = (float)g->iseg[k][q];
    }
    g->nseg = n + g->nint;

    /* light: DGC:171-172 / HMC:18 / XOC:18 / FOC:18-19 / SHC:18-19; MC:143-144 */
    g->has_light = !(c->mission == OR_HOMING || c->mission == OR_XOR);
    g->light[0] = 0.0f;
    g->light[1] = (c->profile == OR_STANDALONE) ? -1.4f : -1.5f;

    static const double div[8] = {10.5884, 3.5999, 2.0, 1.2, 0.8571, 0.6667, 0.5806, 0.5247};
    for (int k = 0; k < 8; k++) {
        float a = (float)(PI_D / div[k]);                               /* ES:28-37 */
        g->cos_a[k] = cosf(a);
        g->sin_a[k] = -sinf(a);                                         /* ES:77 */
    }
    const float deg2rad = (float)(PI_D / 180.0);
    for (int k = 0; k < 4; k++) {
        float a = (45.0f + 90.0f * k) * deg2rad;                        /* ES:40-41 */
        g->rab_cos[k] = cosf(a);
        g->rab_sin[k] = sinf(a);
    }
}

/* ------------------------------------------------------------------------ */
/*  libm conditioning probe. The reference evaluates cos/sin/atan2/exp with  */
/*  torch's CPU kernels (SLEEF), this oracle with glibc and the HIP kernel   */
/*  with ocml; each is within ~1 ulp of the true value but they differ. The  */
/*  parity envelope (tests/parity.py) re-runs the oracle with every such     */
/*  result nudged by +-g_lm_ulps ulp to measure how far a step's outputs can */
/*  move under that freedom. 0 (the default) = plain libm.                   */
/* ------------------------------------------------------------------------ */
/*  sin and cos can also be nudged independently (or_set_libm_perturb3): two  */
/*  implementations' sincos may round the pair in opposite directions.       */
static int g_lm_sin = 0, g_lm_cos = 0, g_lm_other = 0;
void or_set_libm_perturb(int ulps) { g_lm_sin = g_lm_cos = g_lm_other = ulps; }
void or_set_libm_perturb3(int sin_ulps, int cos_ulps, int other_ulps) {
    g_lm_sin = sin_ulps;
    g_lm_cos = cos_ulps;
    g_lm_other = other_ulps;
}
static inline float lm_nudge(float v, int ulps) {
    for (int k = 0; k < ulps; k++) v = nextafterf(v, INFINITY);
    for (int k = 0; k < -ulps; k++) v = nextafterf(v, -INFINITY);
    return v;
}
static inline float lm_cos(float a) { return lm_nudge(cosf(a), g_lm_cos); }
static inline float lm_sin(float a) { return lm_nudge(sinf(a), g_lm_sin); }
static inline float lm_atan2(float y, float x) { return lm_nudge(atan2f(y, x), g_lm_other); }
static inline float lm_exp(float a) { return lm_nudge(expf(a), g_lm_other); }

/* physical constants (DGC:122-137, 179; MC:118-121, 185-189) */
#define R_ROBOT 0.035
#define MAX_SPEED 0.16f
#define WHEELBASE 0.055f
#define DT 0.1f
#define PROX_RANGE 0.10f
#define RAB_RANGE 0.60f
#define RAB_LOSS 0.85f
#define UNITY 0.10f
#define LIGHT_THR 0.2f
#define LIGHT_INT 1000.0f
#define ALPHA 5.0f
#define PROX_THR 0.1f

static inline float sgnf(float v) { return (v > 0.0f) ? 1.0f : ((v < 0.0f) ? -1.0f : 0.0f); }
static inline float clampf(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }

/* ------------------------------------------------------------------------ */
/*  Ground colour (0 black, 0.5 grey, 1 white) per mission and profile      */
/* ------------------------------------------------------------------------ */
static float ground(const or_cfg* c, const geom* g, float x, float y) {
    float col = 0.5f;
    switch (c->mission) {
    case OR_HOMING: {                                                   /* HM:76-85, MC:311-313 */
        float dx = x - 0.0f, dy = y - (-0.70f);
        if (dx * dx + dy * dy <= (float)(0.30 * 0.30)) col = 0.0f;
        break;
    }
    case OR_XOR: {                                                      /* XO:110-124, MC:306-309 */
        for (int t = 0; t < 2; t++) {
            float dx = x - (t ? 0.50f : -0.50f), dy = y - 0.0f;
            if (dx * dx + dy * dy <= (float)(0.30 * 0.30)) col = 0.0f;
        }
        break;
    }
    case OR_FORAGING: {                                                 /* FO:104-125, MC:315-320 */
        for (int t = 0; t < 2; t++) {
            float dx = x - (t ? 0.75f : -0.75f), dy = y - 0.0f;
            if (dx * dx + dy * dy <= (float)(0.15 * 0.15)) col = 0.0f;
        }
        if (y <= (float)g->nest_top) col = 1.0f;
        break;
    }
    case OR_SHELTERING: {                                               /* SH:106-122, MC:331-340 */
        for (int t = 0; t < 2; t++) {
            float dx = x - (t ? 0.80f : -0.80f), dy = y - 0.0f;
            if (dx * dx + dy * dy <= (float)(0.30 * 0.30)) col = 0.0f;
        }
        if (x >= (float)g->shelter[0] && x <= (float)g->shelter[1] &&
            y >= (float)g->shelter[2] && y <= (float)g->shelter[3]) col = 1.0f;
        break;
    }
    default: {                                                          /* DG:707-750, MC:290-304 */
        if (fabsf(x) < (float)g->gate_hw && y > (float)g->gate_south && y < (float)g->corr_south) col = 1.0f;
        if (fabsf(x) < (float)g->corr_hw && y >= (float)g->corr_south && y < (float)g->ni) col = 0.0f;
        break;
    }
    }
    return col;
}

static int in_nest(const geom* g, float y) { return y <= (float)g->nest_top; }

/* ------------------------------------------------------------------------ */
/*  Collisions                                                              */
/* ------------------------------------------------------------------------ */

/* DG:1048-1078 — Jacobi sum of all penetrating faces. */
static void walls_dg(const or_cfg* c, const geom* g, float* pos, int e) {
    const float r = (float)(R_ROBOT + 0.5 * 0.01 + 1e-4);
    for (int i = 0; i < c->N; i++) {
        float* p = pos + ((size_t)e * c->N + i) * 2;
        float tx = 0.0f, ty = 0.0f;
        for (int k = 0; k < 12; k++) {
            float dx = p[0] - g->face_p[k][0], dy = p[1] - g->face_p[k][1];
            float sd = dx * g->face_n[k][0] + dy * g->face_n[k][1];
            float pen = r - sd;
            pen = pen * (pen > 0.0f ? 1.0f : 0.0f);
            tx += pen * g->face_n[k][0];
            ty += pen * g->face_n[k][1];
        }
        p[0] = p[0] + tx;
        p[1] = p[1] + ty;
    }
}

/* MC:531-553 — sequential per face, clearance = robot radius. */
static void walls_mc(const or_cfg* c, const geom* g, float* pos, int e) {
    const float r = (float)R_ROBOT;
    for (int k = 0; k < 12; k++) {
        for (int i = 0; i < c->N; i++) {
            float* p = pos + ((size_t)e * c->N + i) * 2;
            float dx = p[0] - g->mcf_p[k][0], dy = p[1] - g->mcf_p[k][1];
            float sd = dx * g->mcf_n[k][0] + dy * g->mcf_n[k][1];
            float pen = r - sd;
            if (pen > 0.0f) {
                p[0] += pen * g->mcf_n[k][0];
                p[1] += pen * g->mcf_n[k][1];
            }
        }
    }
}

/* DG:1080-1112 / MC:555-571 — Jacobi pairwise half-overlap push over i<j. */
static void robots_push(const or_cfg* c, float* pos, int e) {
    const int N = c->N;
    const float md = (float)(2 * R_ROBOT);
    float* P = pos + (size_t)e * N * 2;
    float rowx[64], rowy[64], colx[64], coly[64];
    for (int i = 0; i < N; i++) rowx[i] = rowy[i] = colx[i] = coly[i] = 0.0f;
    for (int i = 0; i < N; i++) {
        for (int j = 0; j < N; j++) {
            float dx = P[2 * i] - P[2 * j], dy = P[2 * i + 1] - P[2 * j + 1];
            float dist = sqrtf(dx * dx + dy * dy + 1e-8f);
            float ov = md - dist;
            ov = ov < 0.0f ? 0.0f : ov;
            ov = ov * (j > i ? 1.0f : 0.0f);
            float nx = dx / (dist + 1e-8f), ny = dy / (dist + 1e-8f);
            float px = ov * nx * 0.5f, py = ov * ny * 0.5f;
            rowx[i] += px; rowy[i] += py;   /* sum(dim=2) */
            colx[j] += px; coly[j] += py;   /* sum(dim=1) */
        }
    }
    for (int i = 0; i < N; i++) {
        P[2 * i] = (P[2 * i] + rowx[i]) - colx[i];
        P[2 * i + 1] = (P[2 * i + 1] + rowy[i]) - coly[i];
    }
}

/* DG:658-705 (DirGate, and XOR which does not override it) */
static void gate_dg(const or_cfg* c, const geom* g, float* pos, int e) {
    const float r = (float)R_ROBOT;
    const float hw = (float)g->corr_hw;
    const float gs = (float)g->gate_south, top = (float)(g->gate_south + g->side_wall_len);
    for (int i = 0; i < c->N; i++) {
        float* p = pos + ((size_t)e * c->N + i) * 2;
        float py = p[1];
        int in_y = (py > gs) && (py < top);
        float px = p[0];
        float dxl = px - (-hw);
        float penl = r - fabsf(dxl);
        if (penl > 0.0f && in_y && px < 0.0f) {
            float s = sgnf(dxl);
            if (s == 0.0f) s = -1.0f;
            p[0] = (float)(-g->corr_hw) + s * r;
        }
        px = p[0];
        float dxr = px - hw;
        float penr = r - fabsf(dxr);
        if (penr > 0.0f && in_y && px > 0.0f) {
            float s = sgnf(dxr);
            if (s == 0.0f) s = 1.0f;
            p[0] = hw + s * r;
        }
    }
}

/* SH:124-155 / MC:471-496 */
static void gate_shelter(const or_cfg* c, const geom* g, float* pos, int e) {
    const double r = R_ROBOT, t = 0.03;
    const double l = g->shelter[0], rt = g->shelter[1], b = g->shelter[2], tp = g->shelter[3];
    const float half = (float)(r + t / 2);
    for (int i = 0; i < c->N; i++) {
        float* p = pos + ((size_t)e * c->N + i) * 2;
        float py = p[1];
        int vy = (py > (float)(b - r)) && (py < (float)(tp + r));
        for (int w = 0; w < 2; w++) {
            double x0 = w ? rt : l;
            float dx = p[0] - (float)x0;
            if (fabsf(dx) < half && vy) {
                float s = sgnf(dx);
                if (s == 0.0f) s = 1.0f;
                p[0] = (float)x0 + s * half;
            }
        }
        float px = p[0];
        py = p[1];
        int hx = (px > (float)(l - r)) && (px < (float)(rt + r));
        float dy = py - (float)tp;
        if (fabsf(dy) < half && hx) {
            float s = sgnf(dy);
            if (s == 0.0f) s = 1.0f;
            p[1] = (float)tp + s * half;
        }
    }
}

static void gate_walls(const or_cfg* c, const geom* g, float* pos, int e) {
    if (c->profile == OR_ISAAC) {
        /* HM:32-33 and FO:42-43 override to no-op; XO does not (DG version runs). */
        if (c->mission == OR_DGT || c->mission == OR_XOR) gate_dg(c, g, pos, e);
        else if (c->mission == OR_SHELTERING) gate_shelter(c, g, pos, e);
    } else {
        /* MC:469-470 no-op for xor/homing/foraging */
        if (c->mission == OR_DGT) gate_dg(c, g, pos, e);
        else if (c->mission == OR_SHELTERING) gate_shelter(c, g, pos, e);
    }
}

/* DG:898-974 */
static void anti_tunnel(const or_cfg* c, const geom* g, float* pos, const float* prev, int e) {
    if (g->nint == 0) return;
    const float clearance = (float)(R_ROBOT + 0.5 * (c->mission == OR_SHELTERING ? 0.03 : 0.0) + 1e-4);
    const float eps = 1e-8f;
    for (int k = 0; k < g->nint; k++) {
        double ax = g->iseg[k][0], ay = g->iseg[k][1], bx = g->iseg[k][2], by = g->iseg[k][3];
        double abx = bx - ax, aby = by - ay, lsq = abx * abx + aby * aby;
        if (lsq <= 1e-8) continue;
        double len = sqrt(lsq);
        float nx = (float)(-aby / len), ny = (float)(abx / len);
        float ancx = (float)ax, ancy = (float)ay, tx = (float)abx, ty = (float)aby;
        for (int i = 0; i < c->N; i++) {
            float* p = pos + ((size_t)e * c->N + i) * 2;
            const float* q = prev + (size_t)i * 2;   /* env-local block */
            float prx = q[0] - ancx, pry = q[1] - ancy;
            float crx = p[0] - ancx, cry = p[1] - ancy;
            float ps = prx * nx + pry * ny;
            float cs = crx * nx + cry * ny;
            float den = ps - cs;
            float sden = fabsf(den) > eps ? den : 1.0f;
            float st = fabsf(den) > eps ? ps / sden : 0.0f;
            float ix = q[0] + (p[0] - q[0]) * st;
            float iy = q[1] + (p[1] - q[1]) * st;
            float wu = ((ix - ancx) * tx + (iy - ancy) * ty) / (float)lsq;
            int crossed = (ps * cs < 0.0f) && (st >= 0.0f) && (st <= 1.0f) && (wu >= 0.0f) && (wu <= 1.0f);
            if (crossed) {
                float side = sgnf(ps);
                if (side == 0.0f) side = -sgnf(cs);
                if (side == 0.0f) side = 1.0f;
                float desired = side * clearance;
                float corr = desired - cs;
                p[0] = p[0] + corr * nx;
                p[1] = p[1] + corr * ny;
            }
        }
    }
}

/* DG:976-1046 */
static void capsules(const or_cfg* c, const geom* g, float* pos, const float* prev, int e) {
    if (g->nint == 0) return;
    const double thick = (c->mission == OR_SHELTERING) ? 0.03 : 0.01;
    const float clearance = (float)(R_ROBOT + 0.5 * thick + 1e-4);
    const float eps = 1e-8f;
    for (int k = 0; k < g->nint; k++) {
        double ax = g->iseg[k][0], ay = g->iseg[k][1], bx = g->iseg[k][2], by = g->iseg[k][3];
        double abx = bx - ax, aby = by - ay, lsq = abx * abx + aby * aby;
        if (lsq <= 1e-8) continue;
        double len = sqrt(lsq);
        float nx = (float)(-aby / len), ny = (float)(abx / len);
        float ancx = (float)ax, ancy = (float)ay, tx = (float)abx, ty = (float)aby;
        for (int i = 0; i < c->N; i++) {
            float* p = pos + ((size_t)e * c->N + i) * 2;
            float rx = p[0] - ancx, ry = p[1] - ancy;
            float u = (rx * tx + ry * ty) / (float)lsq;
            float uc = clampf(u, 0.0f, 1.0f);
            float clx = ancx + uc * tx, cly = ancy + uc * ty;
            float dx = p[0] - clx, dy = p[1] - cly;
            float raw = sqrtf(dx * dx + dy * dy);
            float dist = raw < eps ? eps : raw;
            float cs = rx * nx + ry * ny;
            float side;
            if (prev) {
                const float* q = prev + (size_t)i * 2;   /* env-local block */
                float qx = q[0] - ancx, qy = q[1] - ancy;
                side = sgnf(qx * nx + qy * ny);
                if (side == 0.0f) side = sgnf(cs);
            } else {
                side = sgnf(cs);
            }
            if (side == 0.0f) side = 1.0f;
            float sdx = side * nx, sdy = side * ny;
            float rdx = raw > eps ? dx / dist : sdx;
            float rdy = raw > eps ? dy / dist : sdy;
            int on_span = (u >= 0.0f) && (u <= 1.0f);
            float pdx = on_span ? sdx : rdx, pdy = on_span ? sdy : rdy;
            float pen = clearance - dist;
            if (pen > 0.0f) {
                float pc = pen < 0.0f ? 0.0f : pen;
                p[0] = p[0] + pc * pdx;
                p[1] = p[1] + pc * pdy;
            }
        }
    }
}

/* DG:874-896; prev = env-local (N,2) block or NULL */
static void resolve_collisions(const or_cfg* c, const geom* g, float* pos, const float* prev, int e) {
    const int N = c->N;
    float before[128];
    walls_dg(c, g, pos, e);
    if (prev) anti_tunnel(c, g, pos, prev, e);
    capsules(c, g, pos, prev, e);
    gate_walls(c, g, pos, e);
    for (int it = 0; it < 4; it++) {                                   /* DGC:127 */
        memcpy(before, pos + (size_t)e * N * 2, sizeof(float) * 2 * N);
        robots_push(c, pos, e);
        walls_dg(c, g, pos, e);
        anti_tunnel(c, g, pos, before, e);
        capsules(c, g, pos, before, e);
        gate_walls(c, g, pos, e);
    }
    walls_dg(c, g, pos, e);
    if (prev) anti_tunnel(c, g, pos, prev, e);
    capsules(c, g, pos, prev, e);
    gate_walls(c, g, pos, e);
}

/* ------------------------------------------------------------------------ */
/*  Sensors (ES)                                                            */
/* ------------------------------------------------------------------------ */
typedef struct {
    float prox8[8], prox_value, prox_angle;
    float light8[8], light_value, light_angle;
    float ztilde, rab4[4], attr_x, attr_y;
} bundle;

/* ES:85-142 with ES:184-242 and ES:244-293 */
static void proximity(const or_cfg* c, const geom* g, const float* pos, const float* yaw, int e, int i, bundle* b) {
    const int N = c->N;
    const float* P = pos + (size_t)e * N * 2;
    float cy = lm_cos(yaw[(size_t)e * N + i]), sy = lm_sin(yaw[(size_t)e * N + i]);
    float ox = P[2 * i], oy = P[2 * i + 1];
    float rdx[8], rdy[8], rd[8];
    for (int k = 0; k < 8; k++) {
        rdx[k] = g->cos_a[k] * cy - g->sin_a[k] * sy;
        rdy[k] = g->cos_a[k] * sy + g->sin_a[k] * cy;
        rd[k] = 0.0f;
    }
    for (int k = 0; k < 8; k++) {
        float segmax = 0.0f;
        for (int s = 0; s < g->nseg; s++) {
            float ax = g->seg[s][0], ay = g->seg[s][1];
            float sx = g->seg[s][2] - ax, sy2 = g->seg[s][3] - ay;
            float den = rdx[k] * sy2 - rdy[k] * sx;
            int valid = fabsf(den) > 1e-8f;
            float t = ((ax - ox) * sy2 - (ay - oy) * sx) / (den + 1e-12f);
            float u = ((ax - ox) * rdy[k] - (ay - oy) * rdx[k]) / (den + 1e-12f);
            int hit = valid && t >= 0.0f && t <= PROX_RANGE && u >= 0.0f && u <= 1.0f;
            float nr = hit ? 1.0f - t / PROX_RANGE : 0.0f;
            if (s == 0 || nr > segmax) segmax = nr;
        }
        rd[k] = rd[k] > segmax ? rd[k] : segmax;
    }
    const float r2 = (float)(R_ROBOT * R_ROBOT);
    for (int k = 0; k < 8; k++) {
        float rmax = 0.0f;
        for (int j = 0; j < N; j++) {
            float dx = P[2 * j] - ox, dy = P[2 * j + 1] - oy;
            float dsq = dx * dx + dy * dy;
            float proj = rdx[k] * dx + rdy[k] * dy;
            float csq = dsq - proj * proj;
            float hc = r2 - csq;
            hc = sqrtf(hc < 0.0f ? 0.0f : hc);
            float hd = proj - hc;
            hd = hd < 0.0f ? 0.0f : hd;
            int hit = (proj > 0.0f) && (csq <= r2) && (hd <= PROX_RANGE) && (j != i);
            float rv = clampf(1.0f - hd / PROX_RANGE, 0.0f, 1.0f);
            float nr = hit ? rv : 0.0f;
            if (j == 0 || nr > rmax) rmax = nr;
        }
        rd[k] = rd[k] > rmax ? rd[k] : rmax;
    }
    float sx = 0.0f, sy3 = 0.0f;
    for (int k = 0; k < 8; k++) {
        b->prox8[k] = rd[k];
        sx += rd[k] * g->cos_a[k];
        sy3 += rd[k] * g->sin_a[k];
    }
    float mag = sqrtf(sx * sx + sy3 * sy3);
    b->prox_value = mag > 1.0f ? 1.0f : mag;
    b->prox_angle = lm_atan2(sy3, sx);
}

/* ES:299-356 */
static void light(const or_cfg* c, const geom* g, const float* pos, const float* yaw, int e, int i, bundle* b) {
    if (!g->has_light) {                                                /* DG:353-362 */
        for (int k = 0; k < 8; k++) b->light8[k] = 0.0f;
        b->light_value = 0.0f;
        b->light_angle = 0.0f;
        return;
    }
    const int N = c->N;
    float x = pos[((size_t)e * N + i) * 2], y = pos[((size_t)e * N + i) * 2 + 1];
    float lx = g->light[0] - x, ly = g->light[1] - y;
    float dist = sqrtf(lx * lx + ly * ly + 1e-6f);
    float du = dist / UNITY;
    float base = LIGHT_INT / du;
    float cy = lm_cos(yaw[(size_t)e * N + i]), sy = lm_sin(yaw[(size_t)e * N + i]);
    float nlx = lx / (dist + 1e-8f), nly = ly / (dist + 1e-8f);
    float raw[8], mx = 0.0f, sx = 0.0f, sy2 = 0.0f;
    for (int k = 0; k < 8; k++) {
        float wdx = g->cos_a[k] * cy - g->sin_a[k] * sy;
        float wdy = g->cos_a[k] * sy + g->sin_a[k] * cy;
        float dot = wdx * nlx + wdy * nly;
        dot = dot < 0.0f ? 0.0f : dot;
        raw[k] = base * dot;
        b->light8[k] = clampf(raw[k], 0.0f, 1.0f);
        if (k == 0 || raw[k] > mx) mx = raw[k];
        sx += raw[k] * g->cos_a[k];
        sy2 += raw[k] * g->sin_a[k];
    }
    float ang = lm_atan2(sy2, sx);
    int above = mx > LIGHT_THR;
    b->light_value = above ? mx : 0.0f;
    b->light_angle = above ? ang : 0.0f;
}

/* ES:382-460 and ES:462-501; u = packet-loss uniforms (N*N for env e) */
static void rab(const or_cfg* c, const geom* g, const float* pos, const float* yaw, int e, int i,
                const float* u, bundle* b) {
    const int N = c->N;
    const float* P = pos + (size_t)e * N * 2;
    float cy = lm_cos(yaw[(size_t)e * N + i]), sy = lm_sin(yaw[(size_t)e * N + i]);
    float ox = P[2 * i], oy = P[2 * i + 1];
    float n = 0.0f, wx = 0.0f, wy = 0.0f, axx = 0.0f, ayy = 0.0f;
    for (int j = 0; j < N; j++) {
        float dx = P[2 * j] - ox, dy = P[2 * j + 1] - oy;
        float dist = sqrtf(dx * dx + dy * dy + 1e-8f);
        int inr = (dist < RAB_RANGE) && (j != i);
        /* line of sight against every wall segment */
        float rdx = dx / (dist + 1e-8f), rdy = dy / (dist + 1e-8f);
        int blocked = 0;
        for (int s = 0; s < g->nseg; s++) {
            float ax = g->seg[s][0], ay = g->seg[s][1];
            float sx = g->seg[s][2] - ax, sy2 = g->seg[s][3] - ay;
            float den = rdx * sy2 - rdy * sx;
            int valid = fabsf(den) > 1e-8f;
            float t = ((ax - ox) * sy2 - (ay - oy) * sx) / (den + 1e-12f);
            float uu = ((ax - ox) * rdy - (ay - oy) * rdx) / (den + 1e-12f);
            if (valid && t > 1e-5f && t < dist - 1e-5f && uu >= 0.0f && uu <= 1.0f) blocked = 1;
        }
        inr = inr && !blocked;
        inr = inr && (u[(size_t)i * N + j] >= RAB_LOSS);
        float inf = inr ? 1.0f : 0.0f;
        n += inf;
        float du = dist / UNITY;
        float inv = 1.0f / (du + 1e-8f);
        float bx = dx * cy + dy * sy;
        float by = -dx * sy + dy * cy;
        float br = lm_atan2(by, bx);
        float cb = lm_cos(br), sb = lm_sin(br);
        wx += inv * cb * inf;
        wy += inv * sb * inf;
        float aw = ALPHA / (1.0f + du);
        axx += aw * cb * inf;
        ayy += aw * sb * inf;
    }
    b->ztilde = 1.0f - 2.0f / (1.0f + lm_exp(n));
    for (int k = 0; k < 4; k++) b->rab4[k] = wx * g->rab_cos[k] + wy * g->rab_sin[k];
    b->attr_x = axx;
    b->attr_y = ayy;
}

/* ------------------------------------------------------------------------ */
/*  Behaviour modules (BM)                                                  */
/* ------------------------------------------------------------------------ */

/* BM:50-90 */
static void wheels_from_vector(float dx, float dy, float* l, float* r) {
    int nz = (fabsf(dx) < 1e-5f) && (fabsf(dy) < 1e-5f);
    float ang = lm_atan2(dy, dx);
    if (ang < 0.0f) ang = ang + (float)(2.0 * PI_D);
    float ca = lm_cos(ang);
    int front = ang < (float)PI_D;
    float lv = front ? ca : 1.0f, rv = front ? 1.0f : ca;
    float mv = fabsf(lv) > fabsf(rv) ? fabsf(lv) : fabsf(rv);
    mv = mv < 1e-5f ? 1e-5f : mv;
    float sc = MAX_SPEED / mv;
    lv = lv * sc;
    rv = rv * sc;
    *l = nz ? 0.0f : lv;
    *r = nz ? 0.0f : rv;
}

static int obstacle_front(float pv, float pa) {                        /* BM:245-251 */
    return (pv >= PROX_THR) && (fabsf(pa) <= (float)(PI_D * 0.5));
}
static float turn_dir(float pa) { return pa < 0.0f ? -1.0f : 1.0f; }  /* BM:253-264 */

typedef struct {
    const int32_t* turns;
    const int32_t* present;
    int E, N;
    int err;
    int used[3];
} turn_src;

static int32_t draw_turn(turn_src* ts, int slot, int e, int i) {
    ts->used[slot] = 1;
    if (ts->turns) {
        if (!ts->present || !ts->present[slot]) { ts->err = -2; return 1; }
        return ts->turns[((size_t)slot * ts->E + e) * ts->N + i];
    }
    return mt_randint(1, 5);
}

/* BM:177-574 for one robot; FSM state updated in place. */
static void dispatch_one(or_state* st, size_t idx, int e, int i, int mod,
                         float pv, float pa, float lv_, float la, float rx_, float ry_,
                         float prev_l, float prev_r, turn_src* ts, float* out_l, float* out_r) {
    const float ms = MAX_SPEED;
    float l = 0.0f, r = 0.0f;
    switch (mod) {
    case 0: l = 0.0f; r = 0.0f; break;                                  /* STOP */
    case 1: {                                                           /* BM:266-341 */
        int state = st->ex_state[idx];
        int steps = st->ex_steps[idx];
        float adir = st->ex_dir[idx];
        int walking = state == 0, was = state == 1;
        int trig = walking && obstacle_front(pv, pa);
        if (trig) {
            adir = turn_dir(pa);
            steps = draw_turn(ts, 0, e, i);
            state = 1;
        }
        if (was) steps = steps - 1;
        if (was && steps <= 0) state = 0;
        l = was ? adir * ms : ms;
        r = was ? (-adir) * ms : ms;
        st->ex_state[idx] = state; st->ex_steps[idx] = steps; st->ex_dir[idx] = adir;
        break;
    }
    case 4: case 5: {                                                   /* BM:343-516 */
        int slot = mod == 4 ? 1 : 2;
        int32_t* av = mod == 4 ? st->ph_avoid : st->ap_avoid;
        int32_t* sp = mod == 4 ? st->ph_steps : st->ap_steps;
        float* dr = mod == 4 ? st->ph_dir : st->ap_dir;
        int avoiding = av[idx];
        int steps = sp[idx];
        float dir = dr[idx];
        int was = avoiding;
        if (was) steps = steps - 1;
        if (was && steps <= 0) avoiding = 0;
        int not_av = !was && !avoiding;
        int trig = not_av && obstacle_front(pv, pa);
        if (trig) {
            dir = turn_dir(pa);
            steps = draw_turn(ts, slot, e, i);
            avoiding = 1;
        }
        av[idx] = avoiding; sp[idx] = steps; dr[idx] = dir;
        float lt = dir * ms, rt = (-dir) * ms;
        float lx = lv_ * lm_cos(la), ly = lv_ * lm_sin(la);
        float px = pv * lm_cos(pa), py = pv * lm_sin(pa);
        float vx, vy;
        if (mod == 4) { vx = lx - 0.5f * px; vy = ly - 0.5f * py; }
        else { vx = (-lx) - 0.5f * px; vy = (-ly) - 0.5f * py; }
        float mag = sqrtf(vx * vx + vy * vy);
        if (mag < 0.1f) { vx = 1.0f; vy = 0.0f; }
        float sl, sr;
        wheels_from_vector(vx, vy, &sl, &sr);
        l = was ? lt : sl;
        r = was ? rt : sr;
        if (trig) { l = prev_l; r = prev_r; }
        break;
    }
    case 2: case 3: {                                                   /* BM:518-574 */
        float px = pv * lm_cos(pa), py = pv * lm_sin(pa);
        float vx, vy;
        if (mod == 2) { vx = rx_ - 0.6f * px; vy = ry_ - 0.6f * py; }
        else { vx = (-ALPHA) * rx_ - 0.5f * px; vy = (-ALPHA) * ry_ - 0.5f * py; }
        float mag = sqrtf(vx * vx + vy * vy);
        if (mag < 0.1f) { vx = 1.0f; vy = 0.0f; }
        wheels_from_vector(vx, vy, &l, &r);
        break;
    }
    default: l = 0.0f; r = 0.0f; break;
    }
    *out_l = l;
    *out_r = r;
}

static void fsm_reset(or_state* st, size_t idx) {                      /* BM:161-173 */
    st->ex_state[idx] = 0; st->ex_steps[idx] = 0; st->ex_dir[idx] = 0.0f;
    st->ph_avoid[idx] = 0; st->ph_steps[idx] = 0; st->ph_dir[idx] = 0.0f;
    st->ap_avoid[idx] = 0; st->ap_steps[idx] = 0; st->ap_dir[idx] = 0.0f;
}

/* ------------------------------------------------------------------------ */
/*  Critic state (ES:545-586, DG:1279-1290)                                 */
/* ------------------------------------------------------------------------ */
void or_critic_state(const or_cfg* c, const float* pos, const float* yaw, float* out) {
    for (size_t q = 0; q < (size_t)c->E * c->N; q++) {
        float rx = pos[2 * q] - 0.0f, ry = pos[2 * q + 1] - 0.0f;
        float nrm = sqrtf(rx * rx + ry * ry);
        nrm = nrm < 1e-6f ? 1e-6f : nrm;
        float rho = clampf(nrm / 1.20f, 0.0f, 1.0f);
        float hx = rx / nrm, hy = ry / nrm;
        float ca = hx * 0.0f + hy * 1.0f;
        float sa = hx * 1.0f - hy * 0.0f;
        float cy = lm_cos(yaw[q]), sy = lm_sin(yaw[q]);
        float cb = cy * hx + sy * hy;
        float sb = hx * sy - hy * cy;
        float* o = out + q * 5;
        o[0] = rho; o[1] = ca; o[2] = sa; o[3] = cb; o[4] = sb;
    }
}

/* ------------------------------------------------------------------------ */
/*  Observation assembly (ES:507-539, DG:1118-1148 / MC:425-440)            */
/* ------------------------------------------------------------------------ */
static void sensor_bundle(const or_cfg* c, const geom* g, const float* pos, const float* yaw, int e,
                          const float* rab_u, bundle* out /* N */) {
    for (int i = 0; i < c->N; i++) {
        proximity(c, g, pos, yaw, e, i, &out[i]);
        light(c, g, pos, yaw, e, i, &out[i]);
        rab(c, g, pos, yaw, e, i, rab_u, &out[i]);
    }
}

static void write_obs(const or_cfg* c, const geom* g, const float* pos, int e, const bundle* b, float* obs) {
    for (int i = 0; i < c->N; i++) {
        size_t q = (size_t)e * c->N + i;
        float gr = ground(c, g, pos[2 * q], pos[2 * q + 1]);
        float* o = obs + q * c->obs_dim;
        if (c->obs_dim == 24) {
            for (int k = 0; k < 8; k++) o[k] = b[i].prox8[k];
            for (int k = 0; k < 8; k++) o[8 + k] = b[i].light8[k];
            o[16] = o[17] = o[18] = gr;
            o[19] = b[i].ztilde;
            for (int k = 0; k < 4; k++) o[20 + k] = b[i].rab4[k];
        } else {
            o[0] = o[1] = o[2] = gr;
            o[3] = b[i].ztilde;
        }
    }
}

static void store_cache(const or_cfg* c, or_state* st, int e, const bundle* b) {
    size_t EN = (size_t)c->E * c->N;
    for (int i = 0; i < c->N; i++) {
        size_t q = (size_t)e * c->N + i;
        st->cache[0 * EN + q] = b[i].prox_value;
        st->cache[1 * EN + q] = b[i].prox_angle;
        st->cache[2 * EN + q] = b[i].light_value;
        st->cache[3 * EN + q] = b[i].light_angle;
        st->cache[4 * EN + q] = b[i].attr_x;
        st->cache[5 * EN + q] = b[i].attr_y;
    }
}

static const float* rab_draw(const float* replay, float* scratch, const or_cfg* c, int e) {
    size_t NN = (size_t)c->N * c->N;
    if (replay) return replay + (size_t)e * NN;
    for (size_t k = 0; k < NN; k++) scratch[k] = mt_uniform();
    return scratch;
}

/* ------------------------------------------------------------------------ */
/*  Isaac profile                                                           */
/* ------------------------------------------------------------------------ */

/* DG:1215-1273 (+ FO:140-151) for the envs flagged in `mask` */
static int isaac_reset_envs(const or_cfg* c, const geom* g, or_state* st, const uint8_t* mask,
                            const or_draws* d) {
    const int E = c->E, N = c->N;
    double cx = 0.0, cy = 0.0, sx = 2.4, sy = 2.4, rad = 1.2;           /* DGC:140-144 */
    if (c->mission == OR_HOMING) { cx = 0.0; cy = 0.7; sx = 2.0; sy = 0.6; rad = 0.8; }  /* HMC:19-21 */
    if (c->mission == OR_FORAGING || c->mission == OR_SHELTERING) { sx = 1.8; sy = 1.8; rad = 0.0; }
    const int max_attempts = 100;
    int any = 0;
    for (int e = 0; e < E; e++) {
        if (!mask[e]) continue;
        any = 1;
        st->ep_len[e] = 0;
        st->completed_reward[e] = st->ep_reward[e];
        st->ep_reward[e] = 0.0f;
        for (int i = 0; i < N; i++) {
            size_t q = (size_t)e * N + i;
            int K = d && d->spawn_u ? d->spawn_k : (rad > 0.0 ? max_attempts + 1 : 1);
            float px = 0.0f, py = 0.0f;
            for (int k = 0; k < K; k++) {
                float u0, u1;
                if (d && d->spawn_u) {
                    u0 = d->spawn_u[(((size_t)k * E + e) * N + i) * 2 + 0];
                    u1 = d->spawn_u[(((size_t)k * E + e) * N + i) * 2 + 1];
                } else {
                    u0 = mt_uniform();
                    u1 = mt_uniform();
                }
                if (k > 0) {                       /* DG:1233-1239 rejection loop */
                    float rx = px - (float)cx, ry = py - (float)cy;
                    if (!(sqrtf(rx * rx + ry * ry) > (float)rad)) break;
                }
                px = (float)cx + (u0 - 0.5f) * (float)sx;
                py = (float)cy + (u1 - 0.5f) * (float)sy;
                if (rad <= 0.0) break;
            }
            st->pos[2 * q] = px;
            st->pos[2 * q + 1] = py;
            float uy = (d && d->spawn_yaw_u) ? d->spawn_yaw_u[q] : mt_uniform();
            st->yaw[q] = uy * 2.0f * (float)PI_D - (float)PI_D;
        }
    }
    if (!any) return 0;
    for (int e = 0; e < E; e++) resolve_collisions(c, g, st->pos, NULL, e);   /* DG:1262 (all envs) */
    for (int e = 0; e < E; e++) {
        if (!mask[e]) continue;
        for (int i = 0; i < N; i++) {
            size_t q = (size_t)e * N + i;
            st->prev_ground[q] = ground(c, g, st->pos[2 * q], st->pos[2 * q + 1]);
            fsm_reset(st, q);
            if (c->mission == OR_FORAGING) {
                st->has_food[q] = 0;
                st->prev_in_nest[q] = in_nest(g, st->pos[2 * q + 1]);
            }
        }
    }
    return 0;
}

static float isaac_reward(const or_cfg* c, const geom* g, or_state* st, int e, int is_final) {
    const int N = c->N;
    float rew = 0.0f;
    switch (c->mission) {
    case OR_HOMING: {                                                   /* HM:87-92 */
        float cnt = 0.0f;
        for (int i = 0; i < N; i++) {
            size_t q = (size_t)e * N + i;
            float dx = st->pos[2 * q] - 0.0f, dy = st->pos[2 * q + 1] - (-0.70f);
            cnt += (dx * dx + dy * dy <= (float)(0.30 * 0.30)) ? 1.0f : 0.0f;
        }
        rew = is_final ? cnt : 0.0f;
        break;
    }
    case OR_XOR: {                                                      /* XO:126-131 */
        float cnt[2] = {0.0f, 0.0f};
        for (int i = 0; i < N; i++) {
            size_t q = (size_t)e * N + i;
            for (int t = 0; t < 2; t++) {
                float dx = st->pos[2 * q] - (t ? 0.50f : -0.50f), dy = st->pos[2 * q + 1] - 0.0f;
                cnt[t] += (dx * dx + dy * dy <= (float)(0.30 * 0.30)) ? 1.0f : 0.0f;
            }
        }
        rew = cnt[0] > cnt[1] ? cnt[0] : cnt[1];
        break;
    }
    case OR_FORAGING: {                                                 /* FO:127-138 */
        float cnt = 0.0f;
        for (int i = 0; i < N; i++) {
            size_t q = (size_t)e * N + i;
            float x = st->pos[2 * q], y = st->pos[2 * q + 1];
            int food = 0;
            for (int t = 0; t < 2; t++) {
                float dx = fabsf(x - (t ? 0.75f : -0.75f)), dy = fabsf(y - 0.0f);
                if (dx <= 0.15f && dy <= 0.15f) food = 1;
            }
            int nest = in_nest(g, y);
            int hf = st->has_food[q] | food;
            int arrived = nest && hf;
            cnt += arrived ? 1.0f : 0.0f;
            st->has_food[q] = arrived ? 0 : hf;
            st->prev_in_nest[q] = nest;
        }
        rew = cnt;
        break;
    }
    case OR_SHELTERING: {                                               /* SH:157-160 */
        float cnt = 0.0f;
        for (int i = 0; i < N; i++) {
            size_t q = (size_t)e * N + i;
            float x = st->pos[2 * q], y = st->pos[2 * q + 1];
            cnt += (x >= (float)g->shelter[0] && x <= (float)g->shelter[1] &&
                    y >= (float)g->shelter[2] && y <= (float)g->shelter[3]) ? 1.0f : 0.0f;
        }
        rew = cnt;
        break;
    }
    default: {                                                          /* DG:1154-1194 */
        float kp = 0.0f, km = 0.0f;
        for (int i = 0; i < N; i++) {
            size_t q = (size_t)e * N + i;
            float cur = ground(c, g, st->pos[2 * q], st->pos[2 * q + 1]);
            float prv = st->prev_ground[q];
            kp += (prv < 0.25f && cur > 0.75f) ? 1.0f : 0.0f;
            km += (prv > 0.75f && cur < 0.25f) ? 1.0f : 0.0f;
            st->prev_ground[q] = cur;
        }
        rew = kp - km;
        break;
    }
    }
    return rew;
}

static void drive(const or_cfg* c, or_state* st, int e, const float* L, const float* R) {
    for (int i = 0; i < c->N; i++) {                                    /* ES:592-617, DG:816-826 */
        size_t q = (size_t)e * c->N + i;
        float v = 0.5f * (L[i] + R[i]);
        float om = (R[i] - L[i]) / WHEELBASE;
        float cy = lm_cos(st->yaw[q]), sy = lm_sin(st->yaw[q]);
        float dx = v * cy * DT, dy = v * sy * DT, dyaw = om * DT;
        st->pos[2 * q] += dx;
        st->pos[2 * q + 1] += dy;
        float yw = st->yaw[q] + dyaw;
        st->yaw[q] = lm_atan2(lm_sin(yw), lm_cos(yw));
    }
}

static int step_isaac(const or_cfg* c, const geom* g, or_state* st, const float* act_cont,
                      const int32_t* act_disc, const or_draws* d, float* obs, float* reward, int32_t* trunc) {
    const int E = c->E, N = c->N;
    turn_src ts = {d ? d->turns : NULL, d ? d->turn_present : NULL, E, N, 0, {0, 0, 0}};
    float L[64], R[64], prev[128];
    size_t EN = (size_t)E * N;
    for (int e = 0; e < E; e++) {
        /* _apply_action (DG:761-843), first substep computes wheels */
        for (int i = 0; i < N; i++) {
            size_t q = (size_t)e * N + i;
            if (c->discrete) {
                dispatch_one(st, q, e, i, act_disc[q],
                             st->cache[0 * EN + q], st->cache[1 * EN + q], st->cache[2 * EN + q],
                             st->cache[3 * EN + q], st->cache[4 * EN + q], st->cache[5 * EN + q],
                             st->wheel_l[q], st->wheel_r[q], &ts, &L[i], &R[i]);
            } else {
                L[i] = clampf(act_cont[2 * q], -1.0f, 1.0f) * MAX_SPEED;
                R[i] = clampf(act_cont[2 * q + 1], -1.0f, 1.0f) * MAX_SPEED;
            }
            st->wheel_l[q] = L[i];
            st->wheel_r[q] = R[i];
        }
        for (int sub = 0; sub < (c->decimation > 0 ? c->decimation : 1); sub++) {
            memcpy(prev, st->pos + (size_t)e * N * 2, sizeof(float) * 2 * N);
            drive(c, st, e, L, R);
            walls_dg(c, g, st->pos, e);
            gate_walls(c, g, st->pos, e);
            robots_push(c, st->pos, e);
            resolve_collisions(c, g, st->pos, prev, e);
        }
    }
    if (ts.err) return ts.err;
    uint8_t* mask = (uint8_t*)calloc((size_t)E, 1);
    for (int e = 0; e < E; e++) {
        st->ep_len[e] += 1;
        int tout = st->ep_len[e] >= c->max_len;                         /* DG:1200-1209 */
        mask[e] = (uint8_t)tout;
        if (tout) {
            or_cfg one = *c;
            one.E = 1;
            or_critic_state(&one, st->pos + (size_t)e * N * 2, st->yaw + (size_t)e * N,
                            st->terminal_critic + (size_t)e * N * 5);
        }
        float r = isaac_reward(c, g, st, e, tout);
        st->ep_reward[e] += r;
        reward[e] = r;
        trunc[e] = tout;
    }
    int rc = isaac_reset_envs(c, g, st, mask, d);
    free(mask);
    if (rc) return rc;
    float* scratch = (float*)malloc(sizeof(float) * N * N);
    bundle b[64];
    for (int e = 0; e < E; e++) {                                       /* DG:1118-1148 */
        const float* u = rab_draw(d ? d->rab_u_obs : NULL, scratch, c, e);
        sensor_bundle(c, g, st->pos, st->yaw, e, u, b);
        store_cache(c, st, e, b);
        write_obs(c, g, st->pos, e, b, obs);
    }
    free(scratch);
    return 0;
}

/* Sensor bundle of the current state: fills the cache and the observation. */
int or_observe(const or_cfg* c, or_state* st, const float* rab_u, float* obs) {
    geom g;
    build_geom(c, &g);
    float* scratch = (float*)malloc(sizeof(float) * c->N * c->N);
    bundle b[64];
    for (int e = 0; e < c->E; e++) {
        const float* u = rab_draw(rab_u, scratch, c, e);
        sensor_bundle(c, &g, st->pos, st->yaw, e, u, b);
        store_cache(c, st, e, b);
        write_obs(c, &g, st->pos, e, b, obs);
    }
    free(scratch);
    return 0;
}

/* Test hook: n uniforms from the private MT19937 stream (torch.rand semantics). */
void or_rng_uniform(float* out, int n) {
    for (int k = 0; k < n; k++) out[k] = mt_uniform();
}

int or_reset_idx(const or_cfg* c, or_state* st, const uint8_t* env_mask, const or_draws* d, float* obs) {
    geom g;
    build_geom(c, &g);
    uint8_t* mask = (uint8_t*)malloc((size_t)c->E);
    for (int e = 0; e < c->E; e++) mask[e] = env_mask ? (env_mask[e] != 0) : 1;
    int rc = isaac_reset_envs(c, &g, st, mask, d);
    free(mask);
    if (rc) return rc;
    float* scratch = (float*)malloc(sizeof(float) * c->N * c->N);
    bundle b[64];
    for (int e = 0; e < c->E; e++) {
        const float* u = rab_draw(d ? d->rab_u_obs : NULL, scratch, c, e);
        sensor_bundle(c, &g, st->pos, st->yaw, e, u, b);
        store_cache(c, st, e, b);
        write_obs(c, &g, st->pos, e, b, obs);
    }
    free(scratch);
    return 0;
}

int or_reset_all(const or_cfg* c, or_state* st, const or_draws* d, float* obs) {
    return or_reset_idx(c, st, NULL, d, obs);
}

/* ------------------------------------------------------------------------ */
/*  Standalone profile (MC:355-423 step, MC:245-269 reset, MC:728-757 loop)  */
/* ------------------------------------------------------------------------ */
static float mc_reward(const or_cfg* c, const geom* g, or_state* st, int e) {
    const int N = c->N;
    switch (c->mission) {
    case OR_XOR: {
        float cnt[2] = {0.0f, 0.0f};
        for (int i = 0; i < N; i++) {
            size_t q = (size_t)e * N + i;
            for (int t = 0; t < 2; t++) {
                float dx = st->pos[2 * q] - (t ? 0.50f : -0.50f), dy = st->pos[2 * q + 1] - 0.0f;
                cnt[t] += (dx * dx + dy * dy <= (float)(0.30 * 0.30)) ? 1.0f : 0.0f;
            }
        }
        return cnt[0] > cnt[1] ? cnt[0] : cnt[1];
    }
    case OR_HOMING: {
        int final_step = st->ep_len[e] + 1 >= c->max_len;
        float cnt = 0.0f;
        for (int i = 0; i < N; i++) {
            size_t q = (size_t)e * N + i;
            float dx = st->pos[2 * q] - 0.0f, dy = st->pos[2 * q + 1] - (-0.70f);
            cnt += (dx * dx + dy * dy <= (float)(0.30 * 0.30)) ? 1.0f : 0.0f;
        }
        return final_step ? cnt : 0.0f;
    }
    case OR_FORAGING: {
        float cnt = 0.0f;
        for (int i = 0; i < N; i++) {
            size_t q = (size_t)e * N + i;
            float x = st->pos[2 * q], y = st->pos[2 * q + 1];
            int food = 0;
            for (int t = 0; t < 2; t++) {
                float dx = x - (t ? 0.75f : -0.75f), dy = y - 0.0f;
                if (dx * dx + dy * dy <= (float)(0.15 * 0.15)) food = 1;
            }
            int nest = in_nest(g, y);
            int hf = st->has_food[q] | food;
            int arrived = nest && !st->prev_in_nest[q] && hf;
            cnt += arrived ? 1.0f : 0.0f;
            st->has_food[q] = arrived ? 0 : hf;
            st->prev_in_nest[q] = nest;
        }
        return cnt;
    }
    case OR_SHELTERING: {
        float cnt = 0.0f;
        for (int i = 0; i < N; i++) {
            size_t q = (size_t)e * N + i;
            float x = st->pos[2 * q], y = st->pos[2 * q + 1];
            cnt += (x >= (float)g->shelter[0] && x <= (float)g->shelter[1] &&
                    y >= (float)g->shelter[2] && y <= (float)g->shelter[3]) ? 1.0f : 0.0f;
        }
        return cnt;
    }
    default: {
        float kp = 0.0f, km = 0.0f;
        for (int i = 0; i < N; i++) {
            size_t q = (size_t)e * N + i;
            float cur = ground(c, g, st->pos[2 * q], st->pos[2 * q + 1]);
            float prv = st->prev_ground[q];
            kp += (prv < 0.25f && cur > 0.75f) ? 1.0f : 0.0f;
            km += (prv > 0.75f && cur < 0.25f) ? 1.0f : 0.0f;
            st->prev_ground[q] = cur;
        }
        return kp - km;
    }
    }
}

static void mc_reset_env(const or_cfg* c, const geom* g, or_state* st, int e, const or_draws* d) {
    const int N = c->N;
    const double safe = g->ni - R_ROBOT * 2;                            /* MC:250-251 */
    st->completed_reward[e] = st->ep_reward[e];
    /* draw order in MC: all r, then all th, then all yaw (three torch.rand(N)) */
    float ur[64], ut[64], uy[64];
    for (int k = 0; k < 3; k++) {
        for (int i = 0; i < N; i++) {
            size_t q = (size_t)e * N + i;
            float u = (d && d->spawn_u) ? d->spawn_u[(size_t)k * c->E * N + q] : mt_uniform();
            (k == 0 ? ur : (k == 1 ? ut : uy))[i] = u;
        }
    }
    for (int i = 0; i < N; i++) {
        size_t q = (size_t)e * N + i;
        float r = sqrtf(ur[i]) * (float)safe;
        float th = ut[i] * (float)(c->mission == OR_HOMING ? PI_D : 2 * PI_D);
        float x = r * lm_cos(th), y = r * lm_sin(th);
        if (c->mission == OR_HOMING) y = fabsf(y);
        st->pos[2 * q] = x;
        st->pos[2 * q + 1] = y;
        st->yaw[q] = uy[i] * 2.0f * (float)PI_D - (float)PI_D;
        st->prev_ground[q] = ground(c, g, x, y);
        st->has_food[q] = 0;
        st->prev_in_nest[q] = in_nest(g, y);
        fsm_reset(st, q);
    }
    st->ep_reward[e] = 0.0f;
    st->ep_len[e] = 0;
}

static int step_standalone(const or_cfg* c, const geom* g, or_state* st, const float* act_cont,
                           const int32_t* act_disc, const float* ovr, const or_draws* d,
                           float* obs, float* reward, int32_t* trunc) {
    const int E = c->E, N = c->N;
    turn_src ts = {d ? d->turns : NULL, d ? d->turn_present : NULL, E, N, 0, {0, 0, 0}};
    float* scratch = (float*)malloc(sizeof(float) * N * N);
    bundle b[64];
    float L[64], R[64];
    for (int e = 0; e < E; e++) {
        /* sensors + dispatch on the current state (MC:730-749; previous = zeros) */
        const float* u = rab_draw(d ? d->rab_u_dispatch : NULL, scratch, c, e);
        sensor_bundle(c, g, st->pos, st->yaw, e, u, b);
        for (int i = 0; i < N; i++) {
            size_t q = (size_t)e * N + i;
            if (c->discrete) {
                dispatch_one(st, q, e, i, act_disc[q], b[i].prox_value, b[i].prox_angle,
                             b[i].light_value, b[i].light_angle, b[i].attr_x, b[i].attr_y,
                             0.0f, 0.0f, &ts, &L[i], &R[i]);
            } else {
                L[i] = act_cont[2 * q] * MAX_SPEED;
                R[i] = act_cont[2 * q + 1] * MAX_SPEED;
            }
            if (ovr && !isnan(ovr[2 * q])) { L[i] = ovr[2 * q]; R[i] = ovr[2 * q + 1]; }
            L[i] = clampf(L[i], -MAX_SPEED, MAX_SPEED);                 /* MC:357-358 */
            R[i] = clampf(R[i], -MAX_SPEED, MAX_SPEED);
            st->wheel_l[q] = L[i];
            st->wheel_r[q] = R[i];
        }
        drive(c, st, e, L, R);                                          /* MC:360-366 */
        walls_mc(c, g, st->pos, e);
        gate_walls(c, g, st->pos, e);
        robots_push(c, st->pos, e);
        float r = mc_reward(c, g, st, e);                               /* MC:372-423 */
        st->ep_reward[e] += r;
        st->ep_len[e] += 1;
        reward[e] = r;
        trunc[e] = 0;
        if (st->ep_len[e] >= c->max_len) {                              /* MC:753-754 */
            mc_reset_env(c, g, st, e, d);
            trunc[e] = 1;
        }
    }
    if (ts.err) { free(scratch); return ts.err; }
    for (int e = 0; e < E; e++) {                                       /* MC:757, 425-440 */
        const float* u = rab_draw(d ? d->rab_u_obs : NULL, scratch, c, e);
        sensor_bundle(c, g, st->pos, st->yaw, e, u, b);
        store_cache(c, st, e, b);
        write_obs(c, g, st->pos, e, b, obs);
    }
    free(scratch);
    return 0;
}

int or_step(const or_cfg* c, or_state* st, const float* act_cont, const int32_t* act_disc,
            const float* override_wheels, const or_draws* d, float* obs, float* reward, int32_t* trunc) {
    if (c->N > 64 || c->N < 1 || c->E < 1) return -1;
    geom g;
    build_geom(c, &g);
    if (c->profile == OR_STANDALONE)
        return step_standalone(c, &g, st, act_cont, act_disc, override_wheels, d, obs, reward, trunc);
    return step_isaac(c, &g, st, act_cont, act_disc, d, obs, reward, trunc);
}

/* ---------------------------------------------------------------------------
 *  Draws of the production (Philox) HIP kernel, restated on the host.
 *
 *  The reference draws torch.rand / torch.randint from a Mersenne stream
 *  (ES:420, BM:302-305 / 386-389, DG:1223-1260, MC:252-258); the GPU kernel
 *  draws the same quantities from Philox4x32-10 keyed by the global env id
 *  (swarm_step_impl.h philox4x32 / rng4 / ChunkRng / u01_of5 / u01_of7 /
 *  draw_turn / spawn_isaac / spawn_mc). This function regenerates exactly those
 *  values for one tick, laid out like the replayed reference draws, so the
 *  oracle can check the production kernel element by element: only the source
 *  of the uniforms differs from the reference-pinned replay path.
 * ------------------------------------------------------------------------- */
static void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; r++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        const uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
        c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

/* rng4(L, robot, block, purpose, tick): counter (genv, robot | block << 8 | purpose << 24, tick lo, tick hi) */
static void rng4_host(uint64_t seed, uint32_t genv, uint32_t robot, uint32_t block, uint32_t purpose, uint64_t tick,
                      uint32_t out[4]) {
    out[0] = genv;
    out[1] = robot | (block << 8) | (purpose << 24);
    out[2] = (uint32_t)tick;
    out[3] = (uint32_t)(tick >> 32);
    philox4x32_10(out, (uint32_t)seed, (uint32_t)(seed >> 32));
}

static float u24(uint32_t v) { return (float)(v >> 8) * (1.0f / 16777216.0f); }

static float u_of5(const uint32_t r[4], int w) {
    uint32_t v;
    switch (w) {
    case 0: v = r[0] >> 8; break;
    case 1: v = r[1] >> 8; break;
    case 2: v = r[2] >> 8; break;
    case 3: v = r[3] >> 8; break;
    default: v = (r[0] & 0xFFu) | ((r[1] & 0xFFu) << 8) | ((r[2] & 0xFFu) << 16); break;
    }
    return (float)v * (1.0f / 16777216.0f);
}

static float u_of7(const uint32_t r[4], int w) {
    const uint64_t lo = (uint64_t)r[0] | ((uint64_t)r[1] << 32);
    const uint64_t hi = (uint64_t)r[2] | ((uint64_t)r[3] << 32);
    const int o = 18 * w;
    uint64_t v;
    if (o + 18 <= 64) v = lo >> o;
    else if (o >= 64) v = hi >> (o - 64);
    else v = (lo >> o) | (hi << (64 - o));
    return (float)(uint32_t)(v & 0x3FFFFull) * (1.0f / 262144.0f);
}

/* Packet-loss uniforms (E,N,N) of one purpose: robot i's neighbour j is in part
 * p = j / C (C = ceil(N / parts)); parts = 3 for the step kernel's layout 103,
 * 1 for the reset kernel and layout 1, 4 for layout 4. Entries j == i unused. */
static void philox_rab(uint64_t seed, int64_t env_offset, int E, int N, int parts, uint32_t purpose, uint64_t tick,
                       float* out) {
    const int C = (N + parts - 1) / parts;
    const int k18 = (C == 6 || C == 7);
    for (int e = 0; e < E; e++) {
        const uint32_t genv = (uint32_t)((uint64_t)env_offset + (uint64_t)e);
        for (int i = 0; i < N; i++) {
            float* row = out + ((size_t)e * N + i) * N;
            for (int p = 0; p < parts; p++) {
                const int j0 = p * C, j1 = j0 + C < N ? j0 + C : N;
                uint32_t rb[4] = {0, 0, 0, 0};
                for (int j = j0; j < j1; j++) {
                    const int jj = j - j0;
                    if (k18) {
                        if (jj == 0) rng4_host(seed, genv, (uint32_t)i, (uint32_t)(16 * p), purpose, tick, rb);
                        row[j] = u_of7(rb, jj);
                    } else {
                        if (jj % 5 == 0)
                            rng4_host(seed, genv, (uint32_t)i, (uint32_t)(16 * p + jj / 5), purpose, tick, rb);
                        row[j] = u_of5(rb, jj % 5);
                    }
                }
            }
        }
    }
}

int or_philox_draws(uint64_t seed, int64_t env_offset, int E, int N, int parts, uint64_t tick, int profile,
                    int spawn_k, float* rab_obs, float* rab_dispatch, int32_t* turns, float* spawn_u,
                    float* spawn_yaw_u) {
    enum { P_RAB_OBS = 1, P_RAB_DISPATCH = 2, P_TURN = 3, P_SPAWN = 8, P_SPAWN_YAW = 9 };
    if (E < 1 || N < 1 || N > 64 || parts < 1) return -1;
    if (rab_obs) philox_rab(seed, env_offset, E, N, parts, P_RAB_OBS, tick, rab_obs);
    if (rab_dispatch) philox_rab(seed, env_offset, E, N, parts, P_RAB_DISPATCH, tick, rab_dispatch);
    for (int e = 0; e < E; e++) {
        const uint32_t genv = (uint32_t)((uint64_t)env_offset + (uint64_t)e);
        for (int i = 0; i < N; i++) {
            const size_t q = (size_t)e * N + i, EN = (size_t)E * N;
            uint32_t r[4] = {0, 0, 0, 0};
            if (turns)
                for (int slot = 0; slot < 3; slot++) {
                    rng4_host(seed, genv, (uint32_t)i, 0u, P_TURN + (uint32_t)slot, tick, r);
                    turns[slot * EN + q] = 1 + (int32_t)(r[0] & 3u);
                }
            if (spawn_u && profile == OR_ISAAC) {
                for (int k = 0; k < spawn_k; k++) {
                    if ((k & 1) == 0) rng4_host(seed, genv, (uint32_t)i, (uint32_t)(k >> 1), P_SPAWN, tick, r);
                    spawn_u[((size_t)k * EN + q) * 2 + 0] = u24((k & 1) ? r[2] : r[0]);
                    spawn_u[((size_t)k * EN + q) * 2 + 1] = u24((k & 1) ? r[3] : r[1]);
                }
            } else if (spawn_u) {
                rng4_host(seed, genv, (uint32_t)i, 0u, P_SPAWN, tick, r);
                spawn_u[q] = u24(r[0]);
                spawn_u[EN + q] = u24(r[1]);
                spawn_u[2 * EN + q] = u24(r[2]);
            }
            if (spawn_yaw_u && profile == OR_ISAAC) {
                rng4_host(seed, genv, (uint32_t)i, 0u, P_SPAWN_YAW, tick, r);
                spawn_yaw_u[q] = u24(r[0]);
            }
        }
    }
    return 0;
}

/* test hook: one Philox4x32-10 block (known-answer checks) */
void or_philox4x32(uint32_t* ctr, uint32_t k0, uint32_t k1) { philox4x32_10(ctr, k0, k1); }

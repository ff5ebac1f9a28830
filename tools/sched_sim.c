/* Scheduling simulator (not product code): the block FIM of fim2d.hip on the CPU with K
 * concurrent workers in lock-step rounds, to compare tile-queue policies by work (tile passes)
 * and by time (rounds, one pass each).  Each round, idle workers take tiles from the queue; every
 * held tile runs ONE pass (four Gauss-Seidel quadrant sweeps) against the halo as T held it at
 * the round's start; at the round's end changed cells are written back and the neighbours whose
 * adjacent cells an improved edge undercuts are activated.  A held tile stays (in place) while it
 * changes or was activated meanwhile, up to `passes`; then it is released (re-queued if still
 * changing).  Policies: 0 FIFO (the GPU's queue), 1 smallest entering value first (the key of an
 * activation is the smallest improved edge value), 2 buckets of width delta (then FIFO), 3 the first
 * activation of a never-visited tile (the front) ahead of the FIFO, 4 as 2 but a queued tile keeps the
 * bucket of the activation that queued it (no re-push on a lower key; a released tile that still
 * changes is re-queued with the smallest value it changed to -- the GPU's bucket queue), 5 FIFO with
 * displacement at push (DISP slots from the head; the displaced entry moves to the tail).
 *   gcc -O3 -march=native -o /tmp/sched_sim tools/sched_sim.c -lm
 *   /tmp/sched_sim cost.f32 N policy passes K
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define TS 64
static int N, NT, policy;
static float delta = 0.f;  /* policy 2: bucket width */
static long seq = 0;
static int oneside = 0;  /* 1: each quadrant sweep reads only its upstream neighbours */
static int skipdir = 0;  /* 1: an in-place pass skips the one direction that alone changed the tile last pass */
static int wrap = 0;     /* 1: the skewed sweep's idle tail steps run its rows again (lane l: rows 0..62-l) */
static int earlyx = 0;   /* 1: a quadrant sweep runs by anti-diagonal steps and stops at the first step past the
                          * last step of a dirty cell (changed in the tile's previous pass, or fed by a halo cell
                          * that changed) at which no cell changed (EARLYX; counts steps per pass = max over dirs) */
static long steps_run = 0, steps_full = 0;
static int disp = 8;     /* policy 5: slots scanned from the head at a push (DISP) */
static float *cost, *T, *key_of;
static unsigned char *pend, *held;

static inline float god(float a, float b, float c) {
    float lo = a < b ? a : b, d = fabsf(a - b);
    if (isnan(d)) return INFINITY;
    if (d > c) d = c;
    return lo + 0.5f * (d + sqrtf(2.f * c * c - d * d));
}
static inline float at(int y, int x) { return (y < 0 || x < 0 || y >= N || x >= N) ? INFINITY : T[(size_t)y * N + x]; }

typedef struct { double k; int t; } HE;
static HE* heap; static long hn;
static void hpush(double k, int t) {
    long i = hn++; heap[i].k = k; heap[i].t = t;
    while (i && heap[(i - 1) / 2].k > heap[i].k) { HE x = heap[i]; heap[i] = heap[(i - 1) / 2]; heap[(i - 1) / 2] = x; i = (i - 1) / 2; }
}
static HE hpop(void) {
    HE r = heap[0]; heap[0] = heap[--hn]; long i = 0;
    for (;;) { long l = 2 * i + 1, m = i; if (l < hn && heap[l].k < heap[m].k) m = l; if (l + 1 < hn && heap[l + 1].k < heap[m].k) m = l + 1;
        if (m == i) break; HE x = heap[i]; heap[i] = heap[m]; heap[m] = x; i = m; }
    return r;
}
static int* fifo; static size_t fh, ft, fcap;
static int* ffifo; static size_t ffh, fft;  /* policy 3: first activations of never-visited tiles */
static unsigned char* visited;

static void activate(int t, float k) {
    if (k < key_of[t]) key_of[t] = k;
    if (pend[t]) {
        if (policy == 1 && !held[t]) hpush(key_of[t], t);
        if (policy == 2 && !held[t]) hpush(floor(key_of[t] / delta) * 1e9 + (double)(seq++), t);  /* lazy re-push */
        return;
    }
    pend[t] = 1;
    if (held[t]) return;  /* served in place by its worker */
    if (policy == 1) hpush(key_of[t], t);
    else if (policy == 2 || policy == 4) hpush(floor(key_of[t] / delta) * 1e9 + (double)(seq++), t);  /* bucket, then FIFO */
    else if (policy == 3 && !visited[t]) ffifo[(fft++) % fcap] = t;
    else if (policy == 6 && visited[t] && fh < ft) {
        /* refinement first (the GPU's qslot_put_front with the test inverted): a visited tile's
         * activation takes the next-to-be-taken slot when a backlog exists, its entry to the tail */
        int u = fifo[fh % fcap]; fifo[fh % fcap] = t; fifo[(ft++) % fcap] = u;
    }
    else if (policy == 5) {
        /* FIFO with displacement at push (the GPU's slot CAS): among the next DISP queued entries, the
         * one with the largest key above k gives its slot to t and goes to the tail */
        size_t best = (size_t)-1; float bk = k;
        for (size_t i = fh; i < ft && i < fh + (size_t)disp; ++i) {
            int u = fifo[i % fcap];
            float ku = (pend[u] && !held[u]) ? key_of[u] : -1.f;  /* stale entries are not displaced */
            if (ku > bk) { bk = ku; best = i; }
        }
        if (best != (size_t)-1) { int u = fifo[best % fcap]; fifo[best % fcap] = t; fifo[(ft++) % fcap] = u; }
        else fifo[(ft++) % fcap] = t;
    }
    else fifo[(ft++) % fcap] = t;
}
static int take(void) {
    if (policy == 3)
        while (ffh != fft) { int t = ffifo[(ffh++) % fcap]; if (pend[t] && !held[t]) return t; }
    if (policy && policy != 3 && policy != 5 && policy != 6) {
        while (hn) {
            HE e = hpop();
            if (pend[e.t] && !held[e.t] &&
                (policy == 4 || (policy == 2 ? floor(e.k / 1e9) == floor(key_of[e.t] / delta) : e.k == key_of[e.t]))) return e.t;
        }
        return -1;
    }
    while (fh != ft) { int t = fifo[(fh++) % fcap]; if (pend[t] && !held[t]) return t; }
    return -1;
}

typedef struct { int t, p, last; float kmin; float L[TS + 2][TS + 2], C[TS + 2][TS + 2]; unsigned char D[TS][TS]; } Work;

int main(int argc, char** argv) {
    const char* cf = argv[1]; N = atoi(argv[2]); policy = atoi(argv[3]);
    const int maxp = atoi(argv[4]), K = atoi(argv[5]);
    if (argc > 6) delta = atof(argv[6]);
    if (getenv("ONESIDE")) oneside = 1;
    if (getenv("SKIPDIR")) skipdir = 1;
    if (getenv("WRAP")) wrap = 1;
    if (getenv("EARLYX")) earlyx = 1;
    if (getenv("DISP")) disp = atoi(getenv("DISP"));
    long dsweeps = 0;  /* quadrant sweeps run */
    NT = N / TS;
    const int nt = NT * NT;
    cost = malloc(sizeof(float) * N * N); T = malloc(sizeof(float) * N * N);
    key_of = malloc(sizeof(float) * nt); pend = calloc(nt, 1); held = calloc(nt, 1);
    FILE* f = fopen(cf, "rb"); if (!f || fread(cost, 4, (size_t)N * N, f) != (size_t)N * N) { printf("bad cost\n"); return 1; } fclose(f);
    for (size_t i = 0; i < (size_t)N * N; ++i) T[i] = INFINITY;
    heap = malloc(sizeof(HE) * 256L * nt); fcap = 16L * nt; fifo = malloc(sizeof(int) * fcap);
    ffifo = malloc(sizeof(int) * fcap); visited = calloc(nt, 1);
    for (int i = 0; i < nt; ++i) key_of[i] = INFINITY;
    T[(size_t)(N / 2) * N + N / 2] = 0.f;
    activate((N / 2 / TS) * NT + N / 2 / TS, 0.f);
    Work* W = malloc(sizeof(Work) * K);
    for (int k = 0; k < K; ++k) W[k].t = -1;
    float (*snapE)[4][TS] = malloc(sizeof(float) * 4 * TS * K);  /* unused placeholder */
    (void)snapE;
    long rounds = 0, npass = 0, visits = 0, busy_sum = 0;
    for (;;) {
        /* idle workers take tiles */
        int busy = 0;
        for (int k = 0; k < K; ++k) {
            if (W[k].t < 0) {
                int t = take();
                if (t < 0) continue;
                held[t] = 1; pend[t] = 0; key_of[t] = INFINITY; ++visits; visited[t] = 1;
                W[k].t = t; W[k].p = 0; W[k].last = -1;
                memset(W[k].D, 1, sizeof W[k].D);  /* a (re)staged tile: nothing known, every cell dirty */
                int ty = t / NT, tx = t % NT, y0 = ty * TS, x0 = tx * TS;
                for (int y = -1; y <= TS; ++y)
                    for (int x = -1; x <= TS; ++x) {
                        int in = y >= 0 && y < TS && x >= 0 && x < TS;
                        W[k].L[y + 1][x + 1] = at(y0 + y, x0 + x);
                        W[k].C[y + 1][x + 1] = in ? cost[(size_t)(y0 + y) * N + x0 + x] : INFINITY;
                    }
            } else {
                /* in place: refresh the halo from T as of this round's start */
                int t = W[k].t, y0 = (t / NT) * TS, x0 = (t % NT) * TS;
                if (pend[t]) W[k].last = -1;  /* activated meanwhile: every direction */
                pend[t] = 0; key_of[t] = INFINITY;
                for (int x = -1; x <= TS; ++x) {
                    float n = at(y0 - 1, x0 + x), so = at(y0 + TS, x0 + x);
                    if (x >= 0 && x < TS && n < W[k].L[0][x + 1]) W[k].D[0][x] = 1;  /* fed by a changed halo cell */
                    if (x >= 0 && x < TS && so < W[k].L[TS + 1][x + 1]) W[k].D[TS - 1][x] = 1;
                    W[k].L[0][x + 1] = n; W[k].L[TS + 1][x + 1] = so;
                }
                for (int y = 0; y < TS; ++y) {
                    float w = at(y0 + y, x0 - 1), e = at(y0 + y, x0 + TS);
                    if (w < W[k].L[y + 1][0]) W[k].D[y][0] = 1;
                    if (e < W[k].L[y + 1][TS + 1]) W[k].D[y][TS - 1] = 1;
                    W[k].L[y + 1][0] = w; W[k].L[y + 1][TS + 1] = e;
                }
            }
            ++busy;
        }
        if (!busy) break;
        ++rounds; busy_sum += busy;
        /* one pass per held tile (halo fixed for the round), results buffered in L */
        static unsigned char changed[1 << 16];
        for (int k = 0; k < K; ++k) {
            if (W[k].t < 0) continue;
            ++npass; ++W[k].p;
            float (*L)[TS + 2] = W[k].L, (*C)[TS + 2] = W[k].C;
            int ch = 0, chd[4] = {0, 0, 0, 0};
            if (earlyx) {
                static unsigned char nd[TS][TS];
                memset(nd, 0, sizeof nd);
                int pass_steps = 0;
                for (int d = 0; d < 4; ++d) {
                    int sx = (d & 1) ? -1 : 1, sy = (d & 2) ? -1 : 1, smax = -1;
                    for (int yy = 0; yy < TS; ++yy) for (int xx = 0; xx < TS; ++xx) {
                        int y = sy > 0 ? yy : TS - 1 - yy, x = sx > 0 ? xx : TS - 1 - xx;
                        if (W[k].D[y][x] && xx + yy > smax) smax = xx + yy;
                    }
                    int s = 0;
                    for (; s < 2 * TS - 1; ++s) {
                        int any = 0;
                        for (int xx = 0; xx < TS; ++xx) {
                            int yy = s - xx;
                            if (yy < 0 || yy >= TS) continue;
                            int y = (sy > 0 ? yy : TS - 1 - yy) + 1, x = (sx > 0 ? xx : TS - 1 - xx) + 1;
                            float w = god(L[y][x - sx], L[y - sy][x], C[y][x]);
                            if (w < L[y][x]) { L[y][x] = w; ch = 1; chd[d] = 1; any = 1; nd[y - 1][x - 1] = 1; }
                        }
                        if (s > smax && !any) { ++s; break; }
                    }
                    if (s > pass_steps) pass_steps = s;
                    ++dsweeps;
                }
                steps_run += pass_steps; steps_full += 2 * TS - 1;
                memcpy(W[k].D, nd, sizeof nd);
                changed[k] = ch;
                W[k].last = -1;
                continue;
            }
            for (int d = 0; d < 4; ++d) {
                if (skipdir && W[k].last == d) continue;
                ++dsweeps;
                int sx = (d & 1) ? -1 : 1, sy = (d & 2) ? -1 : 1;
                for (int yy = 0; yy < TS; ++yy) {
                    int y = (sy > 0 ? yy : TS - 1 - yy) + 1;
                    for (int xx = 0; xx < TS; ++xx) {
                        int x = (sx > 0 ? xx : TS - 1 - xx) + 1;
                        float a = oneside ? L[y][x - sx] : fminf(L[y][x - 1], L[y][x + 1]), b = oneside ? L[y - sy][x] : fminf(L[y - 1][x], L[y + 1][x]);
                        float w = god(a, b, C[y][x]);
                        if (w < L[y][x]) { L[y][x] = w; ch = 1; chd[d] = 1; }
                    }
                }
            }
            /* WRAP: the ramp-down steps of the 4 skewed sweeps (lane l idle after step l + 63) run
             * the first 63 - l rows of their column again: the triangle yy + xx <= 62 of each
             * direction's frame (modelled after the four full sweeps) */
            for (int d = 0; wrap && d < 4; ++d) {
                int sx = (d & 1) ? -1 : 1, sy = (d & 2) ? -1 : 1;
                for (int yy = 0; yy < TS - 1; ++yy) {
                    int y = (sy > 0 ? yy : TS - 1 - yy) + 1;
                    for (int xx = 0; xx + yy <= TS - 2; ++xx) {
                        int x = (sx > 0 ? xx : TS - 1 - xx) + 1;
                        float a = oneside ? L[y][x - sx] : fminf(L[y][x - 1], L[y][x + 1]), b = oneside ? L[y - sy][x] : fminf(L[y - 1][x], L[y + 1][x]);
                        float w = god(a, b, C[y][x]);
                        if (w < L[y][x]) { L[y][x] = w; ch = 1; chd[d] = 1; }
                    }
                }
            }
            changed[k] = ch;
            W[k].last = (chd[0] + chd[1] + chd[2] + chd[3] == 1) ? (chd[1] ? 1 : chd[2] ? 2 : chd[3] ? 3 : 0) : -1;
        }
        /* round end: write back, activate, release */
        for (int k = 0; k < K; ++k) {
            if (W[k].t < 0) continue;
            int t = W[k].t, ty = t / NT, tx = t % NT, y0 = ty * TS, x0 = tx * TS;
            float (*L)[TS + 2] = W[k].L;
            float ke[4] = {INFINITY, INFINITY, INFINITY, INFINITY}, kmin = INFINITY;
            for (int y = 0; y < TS; ++y) for (int x = 0; x < TS; ++x) {
                float v = L[y + 1][x + 1];
                float* m = &T[(size_t)(y0 + y) * N + x0 + x];
                if (v < *m) {
                    *m = v; if (v < kmin) kmin = v;
                    if (y == 0 && v < at(y0 - 1, x0 + x) && v < ke[0]) ke[0] = v;
                    if (y == TS - 1 && v < at(y0 + TS, x0 + x) && v < ke[1]) ke[1] = v;
                    if (x == 0 && v < at(y0 + y, x0 - 1) && v < ke[2]) ke[2] = v;
                    if (x == TS - 1 && v < at(y0 + y, x0 + TS) && v < ke[3]) ke[3] = v;
                }
            }
            if (ke[0] < INFINITY && ty > 0) activate(t - NT, ke[0]);
            if (ke[1] < INFINITY && ty + 1 < NT) activate(t + NT, ke[1]);
            if (ke[2] < INFINITY && tx > 0) activate(t - 1, ke[2]);
            if (ke[3] < INFINITY && tx + 1 < NT) activate(t + 1, ke[3]);
            W[k].kmin = kmin;
        }
        for (int k = 0; k < K; ++k) {
            if (W[k].t < 0) continue;
            int t = W[k].t;
            int go_on = changed[k] || pend[t];
            if (go_on && W[k].p < maxp) continue;  /* in place next round */
            held[t] = 0; W[k].t = -1;
            if (go_on) { pend[t] = 0; activate(t, policy == 4 && !getenv("REQ0") ? W[k].kmin : 0.f); }  /* re-queue (key: keep order fair) */
        }
    }
    double s = 0; long fin = 0;
    for (size_t i = 0; i < (size_t)N * N; ++i) if (isfinite(T[i])) { s += T[i]; ++fin; }
    printf("policy %d passes %d K %d: rounds %ld visits %ld passes %ld (%.2f/tile) sweeps %ld avg busy %.0f checksum %.6e finite %ld\n", policy,
           maxp, K, rounds, visits, npass, (double)npass / nt, dsweeps, (double)busy_sum / rounds, s, fin);
    if (earlyx) printf("EARLYX: pass steps run %ld of %ld (%.3f)\n", steps_run, steps_full, (double)steps_run / steps_full);
    return 0;
}

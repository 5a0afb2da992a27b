/*
 * rm_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * Line-by-line CPU restatement of shaders/computeShader.glsl (reference
 * Qirias/OpenGL-RayMarching-in-Compute-Shader).  Every function cites the
 * GLSL lines it follows.  Built with -ffp-contract=off and without fast-math
 * so every + - * / sqrt is one IEEE-754 binary32 operation, in GLSL source
 * order.  GLSL built-ins follow the contract written in DESIGN.md §2:
 *   dot(a,b)      = (a.x*b.x + a.y*b.y) + a.z*b.z        (left to right)
 *   length(v)     = sqrtf(dot(v,v))
 *   normalize(v)  = v * (1.0f / sqrtf(dot(v,v)))         (GLM 0.9.8.5 form)
 *   reflect(I,N)  = I - (2.0f * dot(N,I)) * N
 *   mix(x,y,a)    = x*(1-a) + y*a
 *   min(x,y)      = y < x ? y : x ;  max(x,y) = x < y ? y : x   (GLSL spec)
 *   clamp(x,a,b)  = min(max(x,a),b)
 *   pow(x,y)      = powf (libm)
 *   sin(iTime)    = sinf (libm)
 *   int(f)        = C truncation; % = C remainder
 * The product (librm) never calls this file.
 */
#include "rm_oracle.h"

#include <math.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct v3 {
  float x, y, z;
} v3;

typedef struct tally {
  uint64_t rays, march, reflect, shadow, normals, lights;
} tally;

/* Work counters in the reference's units.  `all` counts everything the GLSL
 * executes; `live` leaves out work whose result provably cannot reach the
 * output: the bounce() iterations after a MATTE prevObject
 * (glsl:189-190 makes them colour no-ops) and the GetNormal of a miss on the
 * last bounce (its normal is never read).  librm's kernels skip exactly that
 * dead work, so their counters equal `live`. */
typedef struct cnt {
  tally live, all;
  int dead;
} cnt;

#define CNT(c, field)                   \
  do {                                  \
    (c)->all.field++;                   \
    if (!(c)->dead) (c)->live.field++;  \
  } while (0)

/* ---- GLSL built-ins under the contract -------------------------------------- */
static inline v3 V(float x, float y, float z) {
  v3 r = {x, y, z};
  return r;
}
static inline v3 add(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 muls(v3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
static inline v3 subs(v3 a, float s) { return V(a.x - s, a.y - s, a.z - s); }
static inline v3 divs(v3 a, float s) { return V(a.x / s, a.y / s, a.z / s); }
static inline float dot3(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static inline float length3(v3 a) { return sqrtf(dot3(a, a)); }
static inline float length2(float x, float y) { return sqrtf(x * x + y * y); }
static inline v3 normalize3(v3 a) { return muls(a, 1.0f / sqrtf(dot3(a, a))); }
static inline float gmin(float x, float y) { return y < x ? y : x; }
static inline float gmax(float x, float y) { return x < y ? y : x; }
static inline float gclamp(float x, float a, float b) { return gmin(gmax(x, a), b); }
static inline v3 vmax0(v3 a) { return V(gmax(a.x, 0.0f), gmax(a.y, 0.0f), gmax(a.z, 0.0f)); }
static inline v3 vabs(v3 a) { return V(fabsf(a.x), fabsf(a.y), fabsf(a.z)); }
/* reflect(I, N) = I - 2.0 * dot(N, I) * N   (GLSL spec) */
static inline v3 reflect3(v3 i, v3 n) { return sub(i, muls(n, 2.0f * dot3(n, i))); }
static inline v3 vpow(v3 a, float e) { return V(powf(a.x, e), powf(a.y, e), powf(a.z, e)); }
static inline v3 L3(const float *p) { return V(p[0], p[1], p[2]); }

#define MAX_STEPS 512      /* glsl:2 */
#define MIN_DIST 0.000001f /* glsl:3 */
#define REFLECTIVE 1.0f    /* glsl:4 */
#define MATTE 0.0f         /* glsl:5 */

/* Uniform-only subexpressions hoisted once per frame (same values the GLSL
 * computes per call): the blend factor sin(iTime)/2+0.5 (glsl:117) and the
 * shadow sharpness k (glsl:185,236). */
typedef struct rctx {
  const rm_uniforms *u;
  float blend;
  float k;
  const rm_primitive *prims; /* runtime scene table (NULL: the GLSL's own scene) */
  int nprims;
} rctx;

static void rctx_init(rctx *r, const rm_uniforms *u) {
  r->u = u;
  r->prims = NULL;
  r->nprims = 0;
  r->blend = sinf(u->iTime) / 2.0f + 0.5f;
  /* 2.0 at glsl:185,236; the hard-shadow extension is k = +inf. */
  r->k = u->shadow_mode == RM_SHADOW_HARD ? INFINITY : 2.0f;
}

typedef struct hit { /* RayHit glsl:39-44 */
  float hitpoint;
  v3 color;
  int id;
  float material;
} hit;

static inline hit H(float d, v3 c, int id, float m) {
  hit h = {d, c, id, m};
  return h;
}

/* GLSL int(float) (glsl:79): truncation toward zero.  GLSL leaves a value outside
 * the int range undefined (and C makes the cast undefined behaviour); the
 * built-in contract takes the gfx950 conversion, v_cvt_i32_f32:
 * saturating, NaN -> 0.  (x86's cvttss2si would give INT_MIN for every such
 * value, whose parity differs from INT_MAX's; found by the sanitizer build.) */
static inline int glsl_int(float x) {
  if (!(x == x)) return 0;
  if (x >= 2147483648.0f) return 2147483647;
  if (x < -2147483648.0f) return -2147483647 - 1;
  return (int)x;
}

/* glsl:77-80  checkers(p) */
static inline v3 checkers(v3 p) {
  return (glsl_int(1000.0f + p.x) % 2 != glsl_int(1000.0f + p.z) % 2) ? V(1.0f, 1.0f, 1.0f)
                                                                       : V(0.2f, 0.2f, 0.2f);
}
/* glsl:83 */
static inline float sdSphere(v3 p, float r) { return length3(p) - r; }
/* glsl:85  dot(p, n.xyz) + n.w */
static inline float sdPlane(v3 p, float nx, float ny, float nz, float nw) {
  return dot3(p, V(nx, ny, nz)) + nw;
}
/* glsl:87-91 */
static inline float sdBox(v3 p, v3 b) {
  v3 d = sub(vabs(p), b);
  return gmin(gmax(d.x, gmax(d.y, d.z)), 0.0f) + length3(vmax0(d));
}
/* glsl:93-96  length(vec2(length(p.xz) - t.x, p.y)) - t.y */
static inline float sdTorus(v3 p, float tx, float ty) {
  return length2(length2(p.x, p.z) - tx, p.y) - ty;
}
/* glsl:98-103 */
static inline float sdCapsule(v3 p, v3 a, v3 b, float r) {
  v3 pa = sub(p, a), ba = sub(b, a);
  float h = gclamp(dot3(pa, ba) / dot3(ba, ba), 0.0f, 1.0f);
  return length3(sub(pa, muls(ba, h))) - r;
}
/* glsl:105  (d1 < d2) ? d1 : d2  — ties keep d2 */
static inline hit opU(hit d1, hit d2) { return (d1.hitpoint < d2.hitpoint) ? d1 : d2; }

/* One runtime-table entry as a RayHit: the GLSL primitive
 * of its type at q = (pos - center) (.xzy when swizzled, as glsl:119 does for
 * the torus), the entry's colour or checkers(pos), id and material. */
static hit table_entry(const rctx *R, const rm_primitive *P, v3 pos) {
  v3 q = sub(pos, L3(P->center));
  if (P->swizzle == RM_SWIZZLE_XZY) q = V(q.x, q.z, q.y);
  const float *a = P->param;
  float d;
  switch (P->type) {
    case RM_PRIM_SPHERE: d = sdSphere(q, a[0]); break;
    case RM_PRIM_BOX: d = sdBox(q, V(a[0], a[1], a[2])); break;
    case RM_PRIM_BLEND: { /* glsl:115-117: mix(Box, Sphere, sin(iTime)/2 + 0.5) */
      float bx = sdBox(q, V(a[0], a[1], a[2]));
      float sp = sdSphere(q, a[3]);
      d = bx * (1.0f - R->blend) + sp * R->blend;
      break;
    }
    case RM_PRIM_TORUS: d = sdTorus(q, a[0], a[1]); break;
    case RM_PRIM_CAPSULE: d = sdCapsule(q, V(a[0], a[1], a[2]), V(a[3], a[4], a[5]), a[6]); break;
    default: d = sdPlane(q, a[0], a[1], a[2], a[3]); break;
  }
  v3 col = P->paint == RM_PAINT_CHECKERS ? checkers(pos) : L3(P->color);
  return H(d, col, P->id, P->material);
}

/* sdf() over a runtime table: the opU chain of glsl:110-122 in table order. */
static hit sdf_table(const rctx *R, v3 pos) {
  hit t = table_entry(R, &R->prims[0], pos);
  for (int k = 1; k < R->nprims; k++) t = opU(t, table_entry(R, &R->prims[k], pos));
  return t;
}

/* glsl:107-123 */
static hit sdf(const rctx *R, v3 pos) {
  if (R->nprims) return sdf_table(R, pos);
  hit t;
  t = H(sdSphere(sub(pos, V(15.0f, 0.0f, -10.0f)), 3.0f), V(0.1804f, 0.6f, 0.2157f), 0,
        REFLECTIVE);
  t = opU(t, H(sdSphere(sub(pos, V(-25.0f, 0.0f, -10.0f)), 3.0f), V(0.0f, 0.851f, 1.0f), 1,
               REFLECTIVE));
  /* Blended shapes, glsl:115-117 */
  hit Box = H(sdBox(sub(pos, V(-5.0f, 0.0f, -10.0f)), V(3.0f, 2.5f, 2.5f)), V(1.0f, 1.0f, 1.0f), 2,
              REFLECTIVE);
  hit Sphere =
      H(sdSphere(sub(pos, V(-5.0f, 0.0f, -10.0f)), 3.0f), V(1.0f, 1.0f, 1.0f), 3, REFLECTIVE);
  float a = R->blend; /* sin(iTime) / 2 + 0.5 */
  float m = Box.hitpoint * (1.0f - a) + Sphere.hitpoint * a; /* mix */
  t = opU(t, H(m, V(0.4863f, 0.3529f, 0.702f), 4, REFLECTIVE));
  /* glsl:119  sdTorus((pos - c).xzy, ...) */
  v3 q = sub(pos, V(-5.0f, 0.0f, 10.0f));
  t = opU(t, H(sdTorus(V(q.x, q.z, q.y), 2.5f, 0.5f), V(0.9137f, 0.549f, 0.0f), 5, REFLECTIVE));
  /* glsl:120 */
  t = opU(t, H(sdCapsule(sub(pos, V(-5.0f, -2.0f, -30.0f)), V(-0.1f, 0.1f, -0.1f),
                         V(2.0f, 4.0f, 2.0f), 1.0f),
               V(0.8f, 0.0902f, 0.4824f), 6, REFLECTIVE));
  /* glsl:121 */
  t = opU(t, H(sdPlane(pos, 0.0f, 1.0f, 0.0f, 5.5f), checkers(pos), 7, MATTE));
  return t;
}

/* glsl:125-142 (RayMarch: tmax 400, MAX_STEPS) and glsl:144-161
 * (reflectedRay: tmax 200, MAX_STEPS/2) share one body. */
static hit march(const rctx *R, v3 ro, v3 rd, int reflected, cnt *c) {
  float t = 0.0f;
  float tmax = reflected ? 200.0f : 400.0f;
  int nmax = reflected ? MAX_STEPS / 2 : MAX_STEPS;
  hit dummy = H(-1.0f, V(0.0f, 0.0f, 0.0f), -1, 1.0f);
  for (int i = 0; i < nmax; i++) {
    hit res = sdf(R, add(ro, muls(rd, t)));
    if (reflected)
      CNT(c, reflect);
    else
      CNT(c, march);
    if (res.hitpoint < (MIN_DIST * t)) return H(t, res.color, res.id, res.material);
    if (res.hitpoint > tmax) return dummy;
    t += res.hitpoint;
  }
  return dummy;
}

/* glsl:278-288 */
static v3 get_normal(const rctx *R, v3 pos, cnt *c) {
  CNT(c, normals);
  float cc = sdf(R, pos).hitpoint;
  v3 v = V(sdf(R, add(pos, V(0.001f, 0.0f, 0.0f))).hitpoint,
           sdf(R, add(pos, V(0.0f, 0.001f, 0.0f))).hitpoint,
           sdf(R, add(pos, V(0.0f, 0.0f, 0.001f))).hitpoint);
  return normalize3(subs(v, cc));
}

/* glsl:253-276 */
static v3 point_light(const rctx *R, v3 color, v3 normal, v3 pos, cnt *c) {
  const rm_uniforms *u = R->u;
  CNT(c, lights);
  const rm_light *L = &u->light;
  v3 lpos = L3(L->position);
  v3 ambient = L3(L->ambient);
  v3 viewDir = normalize3(sub(pos, L3(u->camera.pos)));
  v3 lightDir = normalize3(sub(lpos, pos));
  float NtoL = gmax(dot3(normal, lightDir), 0.0f);
  v3 diffuse = muls(L3(L->diffuse), NtoL);
  v3 reflectDir = reflect3(lightDir, normal);
  float spec = powf(gmax(dot3(viewDir, reflectDir), 0.0f), 32.0f);
  v3 specular = muls(L3(L->specular), spec);
  float distance = length3(sub(lpos, pos));
  float attenuation =
      1.0f / (L->constant + L->linear * distance + L->quadratic * (distance * distance));
  diffuse = muls(diffuse, attenuation);
  ambient = muls(ambient, attenuation);
  specular = muls(specular, attenuation);
  return mul(color, add(add(diffuse, ambient), specular));
}

/* glsl:201-216 */
static float softshadow(const rctx *R, v3 ro, v3 rd, float k, cnt *c) {
  float res = 1.0f;
  float t = 0.0f;
  for (int i = 0; i < 16; i++) {
    hit h = sdf(R, add(ro, muls(rd, t)));
    CNT(c, shadow);
    if (h.hitpoint < 0.001f) return 0.05f;
    res = gmin(res, k * h.hitpoint / t);
    t += h.hitpoint;
  }
  return res;
}

/* glsl:163-199 */
static v3 bounce(const rctx *R, v3 rayDir, v3 pos, v3 normal, v3 color, hit primary,
                 cnt *c) {
  const rm_uniforms *u = R->u;
  hit prevObject = primary;
  float shadow = 1.0f;
  v3 prevColor = primary.color;
  for (int i = 1; i <= u->bounceVar; i++) {
    c->dead = (prevObject.material == MATTE); /* whole iteration is a colour no-op */
    rayDir = reflect3(rayDir, normal);
    hit t = march(R, add(pos, muls(normal, 0.001f)), rayDir, 1, c);
    pos = add(pos, muls(rayDir, t.hitpoint));
    int was_dead = c->dead;
    if (t.hitpoint == -1.0f && i == u->bounceVar) c->dead = 1; /* normal never read */
    normal = get_normal(R, pos, c);
    c->dead = was_dead;
    if (t.hitpoint == -1.0f)
      t.color = subs(V(0.36f, 0.36f, 0.60f), rayDir.y * 0.2f);
    else
      t.color = point_light(R, t.color, normal, pos, c);
    if (t.id == 7 && prevObject.material != MATTE && i < 3) {
      v3 sro = add(pos, muls(normal, 0.02f));
      v3 srd = sub(L3(u->light.position), pos);
      shadow = softshadow(R, sro, srd, R->k, c);
      color = muls(color, shadow / (float)i);
    }
    if (prevObject.material == MATTE)
      continue;
    else
      color = add(color, divs(mul(t.color, prevColor), (float)i));
    prevColor = t.color;
    prevObject = t;
  }
  c->dead = 0;
  return color;
}

/* glsl:218-251 */
static v3 render(const rctx *R, v3 ro, v3 rd, cnt *c) {
  const rm_uniforms *u = R->u;
  v3 color = subs(V(0.30f, 0.36f, 0.60f), rd.y * 0.2f);
  hit t = march(R, ro, rd, 0, c);
  float shadow = 1.0f;
  if (t.hitpoint != -1.0f) {
    v3 pos = add(ro, muls(rd, t.hitpoint));
    v3 normal = get_normal(R, pos, c);
    color = t.color;
    color = point_light(R, color, normal, pos, c);
    if (t.id == 7) {
      v3 sro = add(pos, muls(normal, 0.02f));
      v3 srd = sub(L3(u->light.position), pos);
      shadow = softshadow(R, sro, srd, R->k, c);
      color = muls(color, shadow);
      return vpow(color, 0.4545f);
    }
    if (u->bounceVar > 0) color = bounce(R, rd, pos, normal, color, t, c);
  }
  return vpow(color, 0.4545f);
}

/* glsl:68-74  normalize(uv.x*xAxis + uv.y*yAxis + dir*radians(45)) over vec4
 * The vec4 dot is GLM's (x*x + y*y) + (z*z + w*w) (func_geometric.inl:63-69);
 * with w = 0 (main.cpp:103-106) it equals the left-to-right 3-component dot.
 * radians() is GLM's degrees * float(0.0174532925199432957...) (func_trigonometric.inl:12-17). */
static void cast_ray(const rctx *R, float uvx, float uvy, v3 *ro, v3 *rd, cnt *c) {
  CNT(c, rays);
  const rm_camera *cam = &R->u->camera;
  float P = 45.0f * (float)0.01745329251994329576923690768489;
  float v[4];
  for (int k = 0; k < 4; k++) v[k] = (uvx * cam->xAxis[k] + uvy * cam->yAxis[k]) + cam->dir[k] * P;
  float d = (v[0] * v[0] + v[1] * v[1]) + (v[2] * v[2] + v[3] * v[3]);
  float inv = 1.0f / sqrtf(d);
  *ro = V(cam->pos[0], cam->pos[1], cam->pos[2]);
  *rd = V(v[0] * inv, v[1] * inv, v[2] * inv);
}

/* glsl:291-344  main() for one pixel. */
static void pixel(const rctx *R, int W, int Hh, int px, int py, float out[4], cnt *c) {
  float x = (float)(px * 2 - W) / (float)W; /* glsl:302 */
  float y = (float)(py * 2 - Hh) / (float)Hh; /* glsl:303 */
  v3 ro, rd, col;
  if (R->u->AA) {
    /* glsl:311-335: cumulative offsets, fixed-order sum, then /4 */
    static const float ox[4] = {0.25f, 0.75f, 0.25f, 0.75f};
    static const float oy[4] = {0.25f, 0.25f, 0.75f, 0.75f};
    float acc[3] = {0.0f, 0.0f, 0.0f};
    for (int s = 0; s < 4; s++) {
      x += ox[s] / (float)W;
      y += oy[s] / (float)Hh;
      cast_ray(R, x, y, &ro, &rd, c);
      col = render(R, ro, rd, c);
      acc[0] += col.x;
      acc[1] += col.y;
      acc[2] += col.z;
    }
    out[0] = acc[0] / 4.0f;
    out[1] = acc[1] / 4.0f;
    out[2] = acc[2] / 4.0f;
    out[3] = 4.0f / 4.0f;
  } else {
    cast_ray(R, x, y, &ro, &rd, c);
    col = render(R, ro, rd, c);
    out[0] = col.x;
    out[1] = col.y;
    out[2] = col.z;
    out[3] = 1.0f;
  }
}

/* ---- public entry points ------------------------------------------------------- */
/* RGBA8 quantization round(clamp(c,0,1)*255); NaN maps to 0. */
uint8_t rmo_quantize(float c) {
  float v = (c > 0.0f) ? ((c < 1.0f) ? c : 1.0f) : 0.0f;
  return (uint8_t)(v * 255.0f + 0.5f);
}

int rmo_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

static void tally_add(tally *a, const tally *b) {
  a->rays += b->rays;
  a->march += b->march;
  a->reflect += b->reflect;
  a->shadow += b->shadow;
  a->normals += b->normals;
  a->lights += b->lights;
}

static void tally_out(const tally *t, rm_counters *o) {
  o->rays = t->rays;
  o->march_steps = t->march;
  o->reflect_steps = t->reflect;
  o->shadow_steps = t->shadow;
  o->normals = t->normals;
  o->lights = t->lights;
  o->sdf_evals = t->march + t->reflect + t->shadow + 4 * t->normals;
}

static int render_rows(const rctx *R, int32_t W, int32_t Hh, const int32_t *rows, int32_t nrows,
                       float *rgba32f, uint8_t *rgba8, uint32_t *sdf_counts, rm_counters *counters,
                       rm_counters *full_counters, int32_t nthreads);

int rmo_render(const rm_uniforms *u, int32_t W, int32_t Hh, const int32_t *rows, int32_t nrows,
               float *rgba32f, uint8_t *rgba8, uint32_t *sdf_counts, rm_counters *counters,
               rm_counters *full_counters, int32_t nthreads) {
  if (!u) return -1;
  rctx Rc;
  rctx_init(&Rc, u);
  return render_rows(&Rc, W, Hh, rows, nrows, rgba32f, rgba8, sdf_counts, counters, full_counters,
                     nthreads);
}

int rmo_render_scene(const rm_uniforms *u, const rm_primitive *prims, int32_t nprims, int32_t W,
                     int32_t Hh, const int32_t *rows, int32_t nrows, float *rgba32f,
                     uint8_t *rgba8, uint32_t *sdf_counts, rm_counters *counters,
                     rm_counters *full_counters, int32_t nthreads) {
  if (!u || !prims || nprims < 1 || nprims > RM_MAX_PRIMITIVES) return -1;
  rctx Rc;
  rctx_init(&Rc, u);
  Rc.prims = prims;
  Rc.nprims = nprims;
  return render_rows(&Rc, W, Hh, rows, nrows, rgba32f, rgba8, sdf_counts, counters, full_counters,
                     nthreads);
}

static int render_rows(const rctx *R, int32_t W, int32_t Hh, const int32_t *rows, int32_t nrows,
                       float *rgba32f, uint8_t *rgba8, uint32_t *sdf_counts, rm_counters *counters,
                       rm_counters *full_counters, int32_t nthreads) {
  if (W <= 0 || Hh <= 0) return -1;
  int32_t n = rows ? nrows : Hh;
  if (n < 0) return -1;
  tally live = {0, 0, 0, 0, 0, 0}, all = {0, 0, 0, 0, 0, 0};
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads)
#endif
  {
    tally llive = {0, 0, 0, 0, 0, 0}, lall = {0, 0, 0, 0, 0, 0};
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
    for (int32_t i = 0; i < n; i++) {
      int32_t py = rows ? rows[i] : i;
      for (int32_t px = 0; px < W; px++) {
        cnt pc;
        memset(&pc, 0, sizeof pc);
        float o[4];
        if (py >= 0 && py < Hh) {
          pixel(R, W, Hh, px, py, o, &pc);
        } else {
          o[0] = o[1] = o[2] = o[3] = 0.0f;
        }
        size_t idx = (size_t)i * (size_t)W + (size_t)px;
        if (rgba32f) memcpy(rgba32f + idx * 4, o, sizeof o);
        if (rgba8) {
          rgba8[idx * 4 + 0] = rmo_quantize(o[0]);
          rgba8[idx * 4 + 1] = rmo_quantize(o[1]);
          rgba8[idx * 4 + 2] = rmo_quantize(o[2]);
          rgba8[idx * 4 + 3] = rmo_quantize(o[3]);
        }
        if (sdf_counts)
          sdf_counts[idx] = (uint32_t)(pc.live.march + pc.live.reflect + pc.live.shadow +
                                       4 * pc.live.normals);
        tally_add(&llive, &pc.live);
        tally_add(&lall, &pc.all);
      }
    }
#ifdef _OPENMP
#pragma omp critical
#endif
    {
      tally_add(&live, &llive);
      tally_add(&all, &lall);
    }
  }
  if (counters) tally_out(&live, counters);
  if (full_counters) tally_out(&all, full_counters);
  return 0;
}

#define RCTX(u)    \
  rctx Rc;         \
  rctx_init(&Rc, u); \
  const rctx *R = &Rc

void rmo_sdf(const rm_uniforms *u, const float pos[3], rmo_hit *out) {
  RCTX(u);
  hit h = sdf(R, L3(pos));
  out->hitpoint = h.hitpoint;
  out->color[0] = h.color.x;
  out->color[1] = h.color.y;
  out->color[2] = h.color.z;
  out->id = h.id;
  out->material = h.material;
}

void rmo_raymarch(const rm_uniforms *u, const float ro[3], const float rd[3], int32_t reflected,
                  rmo_hit *out, uint32_t *steps) {
  RCTX(u);
  cnt c;
  memset(&c, 0, sizeof c);
  hit h = march(R, L3(ro), L3(rd), reflected, &c);
  out->hitpoint = h.hitpoint;
  out->color[0] = h.color.x;
  out->color[1] = h.color.y;
  out->color[2] = h.color.z;
  out->id = h.id;
  out->material = h.material;
  if (steps) *steps = (uint32_t)(reflected ? c.all.reflect : c.all.march);
}

void rmo_get_normal(const rm_uniforms *u, const float pos[3], float out[3]) {
  RCTX(u);
  cnt c;
  memset(&c, 0, sizeof c);
  v3 n = get_normal(R, L3(pos), &c);
  out[0] = n.x;
  out[1] = n.y;
  out[2] = n.z;
}

float rmo_softshadow(const rm_uniforms *u, const float ro[3], const float rd[3], float k,
                     uint32_t *steps) {
  RCTX(u);
  cnt c;
  memset(&c, 0, sizeof c);
  float r = softshadow(R, L3(ro), L3(rd), k, &c);
  if (steps) *steps = (uint32_t)c.all.shadow;
  return r;
}

void rmo_point_light(const rm_uniforms *u, const float color[3], const float normal[3],
                     const float pos[3], float out[3]) {
  RCTX(u);
  cnt c;
  memset(&c, 0, sizeof c);
  v3 r = point_light(R, L3(color), L3(normal), L3(pos), &c);
  out[0] = r.x;
  out[1] = r.y;
  out[2] = r.z;
}

void rmo_cast_ray(const rm_uniforms *u, float uvx, float uvy, float ro[3], float rd[3]) {
  RCTX(u);
  cnt c;
  memset(&c, 0, sizeof c);
  v3 o, d;
  cast_ray(R, uvx, uvy, &o, &d, &c);
  ro[0] = o.x;
  ro[1] = o.y;
  ro[2] = o.z;
  rd[0] = d.x;
  rd[1] = d.y;
  rd[2] = d.z;
}

void rmo_render_ray(const rm_uniforms *u, const float ro[3], const float rd[3], float out[3]) {
  RCTX(u);
  cnt c;
  memset(&c, 0, sizeof c);
  v3 r = render(R, L3(ro), L3(rd), &c);
  out[0] = r.x;
  out[1] = r.y;
  out[2] = r.z;
}

void rmo_pixel(const rm_uniforms *u, int32_t W, int32_t Hh, int32_t px, int32_t py,
               float out[4]) {
  RCTX(u);
  cnt c;
  memset(&c, 0, sizeof c);
  pixel(R, W, Hh, px, py, out, &c);
}

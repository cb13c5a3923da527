/* The R .Call shim of INTEGRATION.md as a plain C program, compiled with gcc against
 * include/hmsc_amd.h (no R, no Python): reads the hM fields from a model file written by
 * tests/capi/model_io.py, fills hmsc_model exactly as the shim does (phylogeny: rhopw and
 * eigen(C); spatial 'Full' levels: alphapw and the unit-ordered coordinates), then runs
 * hmsc_create -> hmsc_init_state -> hmsc_run and writes the recorded samples.
 *
 *   shim_run model.bin out.bin seed mask transient samples
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hmsc_amd.h"

typedef struct {
  char name[64];
  int kind; /* 0 double, 1 int32 */
  int64_t n;
  void* data;
} rec_t;

static rec_t recs[128];
static int nrec = 0;

static int load(const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) return -1;
  int32_t ln;
  while (fread(&ln, 4, 1, f) == 1) {
    rec_t* r = &recs[nrec++];
    if (ln <= 0 || ln >= 64 || nrec > 128) return -2;
    if (fread(r->name, 1, ln, f) != (size_t)ln) return -3;
    r->name[ln] = 0;
    if (fread(&r->kind, 4, 1, f) != 1 || fread(&r->n, 8, 1, f) != 1) return -4;
    const size_t sz = (size_t)r->n * (r->kind ? 4 : 8);
    r->data = malloc(sz ? sz : 8);
    if (sz && fread(r->data, 1, sz, f) != sz) return -5;
  }
  fclose(f);
  return 0;
}

static void* get(const char* name) {
  for (int i = 0; i < nrec; ++i)
    if (!strcmp(recs[i].name, name)) return recs[i].data;
  return NULL;
}
#define DBL(name) ((const double*)get(name))
#define INT(name) ((const int32_t*)get(name))

static void put(FILE* f, const char* name, int kind, int64_t n, const void* data) {
  const int32_t ln = (int32_t)strlen(name);
  fwrite(&ln, 4, 1, f);
  fwrite(name, 1, ln, f);
  fwrite(&kind, 4, 1, f);
  fwrite(&n, 8, 1, f);
  fwrite(data, kind ? 4 : 8, (size_t)n, f);
}

int main(int argc, char** argv) {
  if (argc != 7) {
    fprintf(stderr, "usage: %s model.bin out.bin seed mask transient samples\n", argv[0]);
    return 2;
  }
  if (load(argv[1]) != 0) {
    fprintf(stderr, "cannot read %s\n", argv[1]);
    return 2;
  }
  const uint64_t seed = strtoull(argv[3], NULL, 10);
  const uint32_t mask = (uint32_t)strtoul(argv[4], NULL, 10);
  const int transient = atoi(argv[5]), S = atoi(argv[6]);

  /* ---- the shim's marshalling (hmsc_run_chain_R) ---- */
  hmsc_model mod;
  memset(&mod, 0, sizeof mod);
  mod.struct_size = HMSC_MODEL_SIZE;
  const int32_t* dims = INT("dims");
  mod.ny = dims[0], mod.ns = dims[1], mod.nc = dims[2], mod.nt = dims[3], mod.nr = dims[4];
  mod.Y = DBL("Y"), mod.Yraw = DBL("Yraw"), mod.X = DBL("X"), mod.Tr = DBL("Tr");
  mod.Pi = INT("Pi"), mod.np = INT("np"), mod.distr = INT("distr");
  mod.V0 = DBL("V0"), mod.f0 = DBL("f0")[0], mod.mGamma = DBL("mGamma"), mod.UGamma = DBL("UGamma");
  mod.aSigma = DBL("aSigma"), mod.bSigma = DBL("bSigma");
  mod.nu = DBL("nu"), mod.a1 = DBL("a1"), mod.b1 = DBL("b1"), mod.a2 = DBL("a2"), mod.b2 = DBL("b2");
  mod.nfMin = INT("nfMin"), mod.nfMax = INT("nfMax"), mod.sDim = INT("sDim");
  static int32_t xdim[HMSC_MAX_LEVELS];
  mod.xDim = xdim;
  /* phylogeny: rhopw and e = eigen(hM$C, symmetric = TRUE) */
  mod.C = DBL("C");
  if (mod.C) {
    const rec_t* rp = NULL;
    for (int i = 0; i < nrec; ++i)
      if (!strcmp(recs[i].name, "rhopw")) rp = &recs[i];
    mod.nrho = (int32_t)(rp->n / 2);
    mod.rhopw = DBL("rhopw"), mod.C_vectors = DBL("C_vectors"), mod.C_values = DBL("C_values");
  }
  /* spatial 'Full' levels: alphapw and the unit-ordered coordinates (grid built on the device) */
  mod.spatialMethod = INT("spatialMethod"), mod.nalpha = INT("nalpha");
  for (int r = 0; r < mod.nr && r < HMSC_MAX_LEVELS; ++r) {
    char nm[32];
    snprintf(nm, sizeof nm, "alphapw%d", r);
    mod.alphapw[r] = DBL(nm);
    snprintf(nm, sizeof nm, "sCoord%d", r);
    mod.sCoord[r] = DBL(nm);
  }
  mod.nNeighbours = INT("nNeighbours"); /* NNGP levels (NULL when the model has none) */

  hmsc_state* st = NULL;
  if (hmsc_create(&mod, seed, 0, mask, &st)) {
    fprintf(stderr, "hmsc_create: %s\n", hmsc_last_error());
    return 1;
  }
  if (hmsc_init_state(st, mod.nfMin)) {
    fprintf(stderr, "hmsc_init_state: %s\n", hmsc_last_error());
    return 1;
  }
  const int ny = mod.ny, ns = mod.ns, nc = mod.nc, nt = mod.nt, nr = mod.nr;
  hmsc_record rec;
  memset(&rec, 0, sizeof rec);
  rec.Beta = calloc((size_t)S * nc * ns, 8);
  rec.Gamma = calloc((size_t)S * nc * nt, 8);
  rec.iV = calloc((size_t)S * nc * nc, 8);
  rec.iSigma = calloc((size_t)S * ns, 8);
  rec.rho = calloc((size_t)S, 4);
  rec.rec_nf = calloc((size_t)S * (nr > 0 ? nr : 1), 4);
  for (int r = 0; r < nr; ++r) {
    const int nfm = mod.nfMax[r];
    rec.Eta[r] = calloc((size_t)S * mod.np[r] * nfm, 8);
    rec.Lambda[r] = calloc((size_t)S * nfm * ns, 8);
    rec.Psi[r] = calloc((size_t)S * nfm * ns, 8);
    rec.Delta[r] = calloc((size_t)S * nfm, 8);
    rec.Alpha[r] = calloc((size_t)S * nfm, 4);
  }
  int32_t adapt[HMSC_MAX_LEVELS] = {0};
  if (hmsc_run(st, transient, S, 1, adapt, 0, &rec)) {
    fprintf(stderr, "hmsc_run: %s\n", hmsc_last_error());
    return 1;
  }
  hmsc_destroy(st);

  FILE* f = fopen(argv[2], "wb");
  if (!f) return 2;
  put(f, "Beta", 0, (int64_t)S * nc * ns, rec.Beta);
  put(f, "Gamma", 0, (int64_t)S * nc * nt, rec.Gamma);
  put(f, "iV", 0, (int64_t)S * nc * nc, rec.iV);
  put(f, "iSigma", 0, (int64_t)S * ns, rec.iSigma);
  put(f, "rho", 1, S, rec.rho);
  for (int r = 0; r < nr; ++r) {
    char nm[32];
    const int nfm = mod.nfMax[r];
    snprintf(nm, sizeof nm, "Eta%d", r);
    put(f, nm, 0, (int64_t)S * mod.np[r] * nfm, rec.Eta[r]);
    snprintf(nm, sizeof nm, "Lambda%d", r);
    put(f, nm, 0, (int64_t)S * nfm * ns, rec.Lambda[r]);
    snprintf(nm, sizeof nm, "Alpha%d", r);
    put(f, nm, 1, (int64_t)S * nfm, rec.Alpha[r]);
  }
  fclose(f);
  printf("shim_run ok: ny=%d ns=%d nc=%d nr=%d samples=%d\n", ny, ns, nc, nr, S);
  return 0;
}

/* A plain-C host of the drop-in boundary (include/unet_mi355x.h): no Python, no torch in the
 * process -- only libunet_mi355x.so and the HIP runtime it links.  tests/test_c_host_gpu.py writes
 * a state_dict and an input batch as raw files, runs this program, and compares what it writes
 * with the Python binding's forward of the same weights (bitwise: same library, same plan).
 *
 *   unet_c_host --abi                      print UNET_ABI_VERSION of the header and of the library
 *   unet_c_host DIR DTYPE N H W            DIR/manifest.txt, DIR/weights.bin, DIR/x.bin ->
 *                                          DIR/logits.bin, DIR/masks.bin, DIR/boxes.bin
 *
 * manifest.txt: first line "n_classes thr0 thr1 thr2 thr3", then one line per state_dict tensor:
 * "name dtype ndim s0 s1 s2 s3 offset nbytes" (dtype 0 = float32, 1 = int64; offset into
 * weights.bin).  x.bin: float32 NCHW [N][3][H][W].  The forward runs twice -- eagerly
 * (unet_forward_boxes on a stream) and as a captured graph (unet_graph_create / launch) -- and the
 * program checks the two agree bit for bit before writing the eager outputs. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "unet_mi355x.h"

#define CHECK(call)                                                                 \
  do {                                                                              \
    int rc_ = (call);                                                               \
    if (rc_ != UNET_OK) {                                                           \
      fprintf(stderr, "%s failed: %d (%s)\n", #call, rc_, unet_last_error());       \
      return 1;                                                                     \
    }                                                                               \
  } while (0)
#define HIP(call)                                                                   \
  do {                                                                              \
    hipError_t e_ = (call);                                                         \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s failed: %s\n", #call, hipGetErrorString(e_));             \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

static void* read_file(const char* dir, const char* name, size_t* size) {
  char path[4096];
  snprintf(path, sizeof path, "%s/%s", dir, name);
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  const long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  void* p = malloc(n > 0 ? (size_t)n : 1);
  if (p && n > 0 && fread(p, 1, (size_t)n, f) != (size_t)n) {
    free(p);
    p = NULL;
  }
  fclose(f);
  if (size) *size = (size_t)n;
  return p;
}

static int write_file(const char* dir, const char* name, const void* p, size_t n) {
  char path[4096];
  snprintf(path, sizeof path, "%s/%s", dir, name);
  FILE* f = fopen(path, "wb");
  if (!f) return 1;
  const size_t w = fwrite(p, 1, n, f);
  fclose(f);
  return w != n;
}

int main(int argc, char** argv) {
  if (argc == 2 && strcmp(argv[1], "--abi") == 0) {
    printf("header %d library %d\n", UNET_ABI_VERSION, unet_abi_version());
    return unet_abi_version() == UNET_ABI_VERSION ? 0 : 1;
  }
  if (argc != 6) {
    fprintf(stderr, "usage: %s DIR DTYPE N H W | --abi\n", argv[0]);
    return 2;
  }
  const char* dir = argv[1];
  const int dtype = atoi(argv[2]), N = atoi(argv[3]), H = atoi(argv[4]), W = atoi(argv[5]);

  /* the state_dict: manifest + one blob of raw tensors */
  char path[4096];
  snprintf(path, sizeof path, "%s/manifest.txt", dir);
  FILE* mf = fopen(path, "r");
  if (!mf) { fprintf(stderr, "no %s\n", path); return 1; }
  unet_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.n_channels = 3;
  cfg.dtype = dtype;
  cfg.device = 0;
  if (fscanf(mf, "%d %f %f %f %f", &cfg.n_classes, &cfg.thresholds[0], &cfg.thresholds[1], &cfg.thresholds[2],
             &cfg.thresholds[3]) != 5) { fprintf(stderr, "bad manifest header\n"); return 1; }
  size_t wbytes = 0;
  uint8_t* blob = (uint8_t*)read_file(dir, "weights.bin", &wbytes);
  if (!blob) { fprintf(stderr, "no weights.bin\n"); return 1; }
  unet_tensor_view views[256];
  char names[256][128];
  int n = 0;
  for (;;) {
    long long s[4], off, nbytes;
    int dt, nd;
    if (fscanf(mf, "%127s %d %d %lld %lld %lld %lld %lld %lld", names[n], &dt, &nd, &s[0], &s[1], &s[2], &s[3],
               &off, &nbytes) != 9) break;
    if (n == 256 || off < 0 || nbytes < 0 || (size_t)(off + nbytes) > wbytes) { fprintf(stderr, "bad manifest\n"); return 1; }
    views[n].name = names[n];
    views[n].data = blob + off;
    views[n].dtype = dt;
    views[n].ndim = nd;
    for (int i = 0; i < 4; ++i) views[n].shape[i] = s[i];
    ++n;
  }
  fclose(mf);

  size_t xbytes = 0;
  float* x_host = (float*)read_file(dir, "x.bin", &xbytes);
  const size_t x_elems = (size_t)N * 3 * H * W;
  if (!x_host || xbytes != x_elems * sizeof(float)) { fprintf(stderr, "x.bin: expected %zu bytes\n", x_elems * 4); return 1; }

  unet_handle* h = NULL;
  CHECK(unet_create(&cfg, &h));
  CHECK(unet_load_weights(h, views, n));
  CHECK(unet_reserve(h, N, H, W));

  const size_t lg_elems = (size_t)N * cfg.n_classes * H * W, box_elems = (size_t)N * cfg.n_classes * 4;
  void *x, *logits, *masks, *boxes, *logits2, *masks2, *boxes2;
  HIP(hipMalloc(&x, x_elems * sizeof(float)));
  HIP(hipMalloc(&logits, lg_elems * sizeof(float)));
  HIP(hipMalloc(&masks, lg_elems));
  HIP(hipMalloc(&boxes, box_elems * sizeof(int32_t)));
  HIP(hipMalloc(&logits2, lg_elems * sizeof(float)));
  HIP(hipMalloc(&masks2, lg_elems));
  HIP(hipMalloc(&boxes2, box_elems * sizeof(int32_t)));
  HIP(hipMemcpy(x, x_host, x_elems * sizeof(float), hipMemcpyHostToDevice));
  hipStream_t stream;
  HIP(hipStreamCreate(&stream));

  /* eager */
  CHECK(unet_forward_boxes(h, x, UNET_LAYOUT_NCHW, UNET_IN_F32, logits, masks, UNET_MASK_U8, (int32_t*)boxes, N, H, W,
                           stream));
  /* captured once, replayed twice */
  unet_graph* g = NULL;
  CHECK(unet_graph_create(h, x, UNET_LAYOUT_NCHW, UNET_IN_F32, logits2, masks2, UNET_MASK_U8, (int32_t*)boxes2, N, H, W,
                          &g));
  CHECK(unet_graph_launch(g, stream));
  CHECK(unet_graph_launch(g, stream));
  HIP(hipStreamSynchronize(stream));

  float* lg = (float*)malloc(lg_elems * sizeof(float));
  float* lg2 = (float*)malloc(lg_elems * sizeof(float));
  uint8_t* mk = (uint8_t*)malloc(lg_elems);
  uint8_t* mk2 = (uint8_t*)malloc(lg_elems);
  int32_t bx[4096], bx2[4096];
  if (!lg || !lg2 || !mk || !mk2 || box_elems > 4096) { fprintf(stderr, "host buffers\n"); return 1; }
  HIP(hipMemcpy(lg, logits, lg_elems * sizeof(float), hipMemcpyDeviceToHost));
  HIP(hipMemcpy(lg2, logits2, lg_elems * sizeof(float), hipMemcpyDeviceToHost));
  HIP(hipMemcpy(mk, masks, lg_elems, hipMemcpyDeviceToHost));
  HIP(hipMemcpy(mk2, masks2, lg_elems, hipMemcpyDeviceToHost));
  HIP(hipMemcpy(bx, boxes, box_elems * sizeof(int32_t), hipMemcpyDeviceToHost));
  HIP(hipMemcpy(bx2, boxes2, box_elems * sizeof(int32_t), hipMemcpyDeviceToHost));
  if (memcmp(lg, lg2, lg_elems * sizeof(float)) || memcmp(mk, mk2, lg_elems) ||
      memcmp(bx, bx2, box_elems * sizeof(int32_t))) {
    fprintf(stderr, "graph replay differs from the eager forward\n");
    return 1;
  }
  if (write_file(dir, "logits.bin", lg, lg_elems * sizeof(float)) || write_file(dir, "masks.bin", mk, lg_elems) ||
      write_file(dir, "boxes.bin", bx, box_elems * sizeof(int32_t))) {
    fprintf(stderr, "cannot write outputs\n");
    return 1;
  }
  CHECK(unet_graph_destroy(g));
  CHECK(unet_destroy(h));
  HIP(hipStreamDestroy(stream));
  hipFree(x); hipFree(logits); hipFree(masks); hipFree(boxes);
  hipFree(logits2); hipFree(masks2); hipFree(boxes2);
  free(lg); free(lg2); free(mk); free(mk2); free(blob); free(x_host);
  printf("ok: %d tensors, N=%d %dx%d, dtype %d, graph == eager\n", n, N, H, W, dtype);
  return 0;
}

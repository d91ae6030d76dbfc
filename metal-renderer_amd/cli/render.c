/*
 * render.c — the C host of the MI355X path tracer: a command-line driver over
 * the C ABI of include/mrt.h (libmrt.so), in place of the reference's app
 * shell (macos/GameViewController.m:10-28 creates the Renderer
 * (renderer/Renderer.h:3-8), sizes it and lets the MTKView call
 * drawInMTKView: once per display refresh; the menu's "Save current image"
 * calls saveCurrentImage).  Here:
 *
 *   -initWithMetalKitView:            mrt_scene_create + mrt_renderer_create
 *   -drawInMTKView: x spp              mrt_renderer_draw_n (1 spp per frame)
 *   -saveCurrentImage                  mrt_renderer_save_image (.pfm / .exr)
 *   window-title stats                 mrt_renderer_stats
 *
 * Multi-GPU (--gpus N): the process forks N ranks BEFORE any
 * libmrt call (no HIP state crosses a fork); rank k renders the 64x64 tiles
 * t % N == k on device k, and the owned tiles reach rank 0 through
 *   --exchange rccl  libmrt's RCCL gather (mrt_comm_*; the 128-byte unique id
 *                    travels from rank 0 to the others over pipes), or
 *   --exchange host  packed tiles through host memory and pipes
 *                    (mrt_renderer_tiles_read / _write; several ranks may then
 *                    share one GPU).
 * Rank 0 writes the image.  Exit status 0 on success, 1 on any error (the
 * message from mrt_last_error on stderr).
 *
 * usage: mrt_render --scene NAME|PATH.obj [--mtl PATH] [--procedural N]
 *                   [--w W] [--h H] [--spp N] [--L L] [--seed S] [--out x.pfm|x.exr]
 *                   [--precise] [--static-noise] [--no-accumulate] [--debug-material]
 *                   [--gpus N] [--device D] [--exchange rccl|host]
 */
#define _GNU_SOURCE
#include <errno.h>
#include <inttypes.h>
#include <limits.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include "mrt.h"

typedef struct {
  const char* scene;
  const char* mtl;
  const char* out;
  const char* exchange;
  uint32_t procedural, width, height, spp, max_path_length, gpus, flags;
  int device;
  uint64_t seed;
} options;

static int die(const char* what) {
  fprintf(stderr, "mrt_render: %s: %s\n", what, mrt_last_error());
  return 1;
}

static void usage(void) {
  fprintf(stderr,
          "usage: mrt_render --scene NAME|PATH.obj [--mtl PATH] [--procedural N] [--w W] [--h H]\n"
          "                  [--spp N] [--L L] [--seed S] [--out x.pfm|x.exr] [--precise]\n"
          "                  [--static-noise] [--no-accumulate] [--debug-material]\n"
          "                  [--gpus N] [--device D] [--exchange rccl|host]\n");
}

/* --scene cornellbox -> <dir of this executable>/../scenes/cornellbox.obj */
static int resolve_scene(const char* name, char* path, size_t n) {
  if (strchr(name, '/') || (strlen(name) > 4 && strcmp(name + strlen(name) - 4, ".obj") == 0)) {
    snprintf(path, n, "%s", name);
    return 0;
  }
  char exe[PATH_MAX / 2];
  const ssize_t k = readlink("/proc/self/exe", exe, sizeof exe - 1);
  if (k <= 0) return -1;
  exe[k] = 0;
  char* slash = strrchr(exe, '/');
  if (!slash) return -1;
  *slash = 0;
  snprintf(path, n, "%s/../scenes/%s.obj", exe, name);
  return 0;
}

static int parse(int argc, char** argv, options* o) {
  *o = (options){.scene = "cornellbox", .out = "render.pfm", .exchange = "rccl", .width = 800, .height = 600,
                 .spp = 16, .max_path_length = 8, .gpus = 1, .seed = 0x6D6574616C2D7274ull};
  for (int i = 1; i < argc; ++i) {
    const char* a = argv[i];
    const char* v = i + 1 < argc ? argv[i + 1] : NULL;
#define VAL(name) (strcmp(a, name) == 0 && v && ++i)
    if (VAL("--scene")) o->scene = v;
    else if (VAL("--mtl")) o->mtl = v;
    else if (VAL("--out")) o->out = v;
    else if (VAL("--exchange")) o->exchange = v;
    else if (VAL("--procedural")) o->procedural = (uint32_t)strtoul(v, NULL, 0);
    else if (VAL("--w")) o->width = (uint32_t)strtoul(v, NULL, 0);
    else if (VAL("--h")) o->height = (uint32_t)strtoul(v, NULL, 0);
    else if (VAL("--spp")) o->spp = (uint32_t)strtoul(v, NULL, 0);
    else if (VAL("--L")) o->max_path_length = (uint32_t)strtoul(v, NULL, 0);
    else if (VAL("--seed")) o->seed = strtoull(v, NULL, 0);
    else if (VAL("--gpus")) o->gpus = (uint32_t)strtoul(v, NULL, 0);
    else if (VAL("--device")) o->device = atoi(v);
    else if (strcmp(a, "--precise") == 0) o->flags |= MRT_FLAG_PRECISE;
    else if (strcmp(a, "--static-noise") == 0) o->flags |= MRT_FLAG_STATIC_NOISE;
    else if (strcmp(a, "--no-accumulate") == 0) o->flags |= MRT_FLAG_NO_ACCUMULATE;
    else if (strcmp(a, "--debug-material") == 0) o->flags |= MRT_FLAG_DEBUG_MATERIAL;
    else {
      usage();
      return -1;
    }
#undef VAL
  }
  if (o->gpus == 0 || o->spp == 0 || (strcmp(o->exchange, "rccl") && strcmp(o->exchange, "host"))) {
    usage();
    return -1;
  }
  return 0;
}

static int write_all(int fd, const void* p, size_t n) {
  const char* c = p;
  while (n) {
    const ssize_t k = write(fd, c, n);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return -1;
    c += k;
    n -= (size_t)k;
  }
  return 0;
}

static int read_all(int fd, void* p, size_t n) {
  char* c = p;
  while (n) {
    const ssize_t k = read(fd, c, n);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return -1;
    c += k;
    n -= (size_t)k;
  }
  return 0;
}

/* One rank of the job.  id_fd: rank 0 writes the RCCL id to the N-1 write
 * ends it owns (to_peer[k]); rank k > 0 reads it from from_root.  tiles:
 * host exchange, rank k > 0 writes its packed tiles to tiles_w, rank 0 reads
 * rank k's from tiles_r[k]. */
static int run_rank(const options* o, uint32_t rank, const int* to_peer, int from_root, const int* tiles_r,
                    int tiles_w) {
  const uint32_t N = o->gpus;
  char obj[PATH_MAX];
  if (resolve_scene(o->scene, obj, sizeof obj)) {
    fprintf(stderr, "mrt_render: cannot resolve scene %s\n", o->scene);
    return 1;
  }
  const int ndev = mrt_device_count();
  if (ndev <= 0) {
    fprintf(stderr, "mrt_render: no HIP device visible\n");
    return 1;
  }
  const int device = N > 1 ? (int)(rank % (uint32_t)ndev) : o->device;
  const int rccl = N > 1 && strcmp(o->exchange, "rccl") == 0;
  mrt_comm* comm = NULL;
  if (rccl) {   /* the communicator first: every rank blocks in it until all have joined */
    unsigned char id[MRT_COMM_ID_BYTES];
    if (rank == 0) {
      if (mrt_comm_unique_id(id, sizeof id)) return die("mrt_comm_unique_id");
      for (uint32_t k = 1; k < N; ++k)
        if (write_all(to_peer[k], id, sizeof id)) return die("send comm id");
    } else if (read_all(from_root, id, sizeof id)) {
      fprintf(stderr, "mrt_render: rank %u: no comm id from rank 0\n", rank);
      return 1;
    }
    if (mrt_comm_create(id, N, rank, device, &comm)) return die("mrt_comm_create");
  }
  mrt_scene_desc sd = {0};
  sd.obj_path = obj;
  sd.mtl_override = o->mtl;
  sd.procedural_triangles = o->procedural;
  sd.procedural_seed = 1;
  sd.device = device;
  mrt_scene* scene = NULL;
  if (mrt_scene_create(&sd, &scene)) return die("mrt_scene_create");
  mrt_renderer_desc rd = {0};
  rd.scene = scene;
  rd.width = o->width;
  rd.height = o->height;
  rd.max_path_length = o->max_path_length;
  rd.seed = o->seed;
  rd.shard_rank = rank;
  rd.shard_count = N;
  rd.flags = o->flags;
  mrt_renderer* r = NULL;
  if (mrt_renderer_create(&rd, &r)) return die("mrt_renderer_create");
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  if (mrt_renderer_draw_n(r, o->spp)) return die("mrt_renderer_draw_n");
  if (rccl) {
    if (mrt_renderer_exchange(r, comm, MRT_EXCHANGE_GATHER)) return die("mrt_renderer_exchange");
  } else if (N > 1) {
    uint64_t floats = 0;
    if (rank > 0) {
      if (mrt_tiles_packed_floats(o->width, o->height, rank, N, &floats)) return die("mrt_tiles_packed_floats");
      float* buf = malloc(floats * sizeof(float) + 1);
      if (!buf || mrt_renderer_tiles_read(r, buf, floats)) return die("mrt_renderer_tiles_read");
      if (write_all(tiles_w, buf, floats * sizeof(float))) return die("send tiles");
      free(buf);
    } else {
      for (uint32_t k = 1; k < N; ++k) {
        if (mrt_tiles_packed_floats(o->width, o->height, k, N, &floats)) return die("mrt_tiles_packed_floats");
        float* buf = malloc(floats * sizeof(float) + 1);
        if (!buf || read_all(tiles_r[k], buf, floats * sizeof(float))) {
          fprintf(stderr, "mrt_render: no tiles from rank %u\n", k);
          return 1;
        }
        if (mrt_renderer_tiles_write(r, k, buf, floats)) return die("mrt_renderer_tiles_write");
        free(buf);
      }
    }
  }
  if (mrt_renderer_sync(r)) return die("mrt_renderer_sync");
  clock_gettime(CLOCK_MONOTONIC, &t1);
  mrt_stats st;
  if (mrt_renderer_stats(r, &st)) return die("mrt_renderer_stats");
  if (rank == 0) {
    if (mrt_renderer_save_image(r, o->out)) return die("mrt_renderer_save_image");
    const double s = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    const double paths = (double)o->width * o->height * o->spp;
    printf("{\"out\": \"%s\", \"width\": %u, \"height\": %u, \"spp\": %u, \"max_path_length\": %u, \"gpus\": %u, "
           "\"exchange\": \"%s\", \"frames\": %" PRIu64 ", \"rank0_paths\": %" PRIu64
           ", \"active_ray_bounces_rank0\": %" PRIu64 ", \"seconds\": %.4f, \"mpaths_per_s\": %.2f}\n",
           o->out, o->width, o->height, o->spp, o->max_path_length, N, N > 1 ? o->exchange : "none",
           st.frame_index, st.paths, st.active_ray_bounces, s, paths / s / 1e6);
    fflush(stdout);
  }
  mrt_renderer_destroy(r);
  mrt_scene_destroy(scene);
  if (comm) mrt_comm_destroy(comm);
  return 0;
}

int main(int argc, char** argv) {
  options o;
  if (parse(argc, argv, &o)) return 2;
  if (mrt_abi_version() != MRT_ABI_VERSION) {
    fprintf(stderr, "mrt_render: libmrt ABI %d, header %d\n", mrt_abi_version(), MRT_ABI_VERSION);
    return 1;
  }
  const uint32_t N = o.gpus;
  if (N == 1) return run_rank(&o, 0, NULL, -1, NULL, -1);
  /* fork the ranks before any HIP call in this process */
  int* id_pipe = calloc(2 * N, sizeof(int));
  int* tile_pipe = calloc(2 * N, sizeof(int));
  pid_t* pid = calloc(N, sizeof(pid_t));
  if (!id_pipe || !tile_pipe || !pid) return 1;
  for (uint32_t k = 1; k < N; ++k)
    if (pipe(id_pipe + 2 * k) || pipe(tile_pipe + 2 * k)) {
      perror("pipe");
      return 1;
    }
  for (uint32_t k = 0; k < N; ++k) {
    pid[k] = fork();
    if (pid[k] < 0) {
      perror("fork");
      return 1;
    }
    if (pid[k] == 0) {
      int* to_peer = calloc(N, sizeof(int));
      int* tiles_r = calloc(N, sizeof(int));
      for (uint32_t j = 1; j < N; ++j) {   /* keep only this rank's pipe ends, so a dead peer reads as EOF */
        to_peer[j] = id_pipe[2 * j + 1];
        tiles_r[j] = tile_pipe[2 * j];
        if (k == 0) {
          close(id_pipe[2 * j]);
          close(tile_pipe[2 * j + 1]);
        } else {
          close(id_pipe[2 * j + 1]);
          close(tile_pipe[2 * j]);
          if (j != k) {
            close(id_pipe[2 * j]);
            close(tile_pipe[2 * j + 1]);
          }
        }
      }
      const int rc = run_rank(&o, k, to_peer, k ? id_pipe[2 * k] : -1, tiles_r, k ? tile_pipe[2 * k + 1] : -1);
      fflush(NULL);
      _exit(rc);
    }
  }
  for (uint32_t k = 1; k < N; ++k) {   /* the parent keeps no pipe ends: a dead rank yields EOF, not a hang */
    close(id_pipe[2 * k]);
    close(id_pipe[2 * k + 1]);
    close(tile_pipe[2 * k]);
    close(tile_pipe[2 * k + 1]);
  }
  int failed = 0;
  for (uint32_t k = 0; k < N; ++k) {
    int status = 0;
    if (waitpid(pid[k], &status, 0) < 0 || !WIFEXITED(status) || WEXITSTATUS(status) != 0) {
      fprintf(stderr, "mrt_render: rank %u failed\n", k);
      failed = 1;
    }
  }
  return failed;
}

// Data-parallel gradient exchange over RCCL (SURVEY §8(b) ptk_comm_init / ptk_comm_allreduce_avg, §8(e)).
//
// Replaces the DDP reducer behind `accelerator.backward` (Stage1/projector_trainer.py:237; accelerate wraps the
// projector in DistributedDataParallel, Stage1/accelerator_setup.py:12-16): one process per GPU, each rank's
// projector grads summed over the ranks and divided by the world size.  RCCL is resolved at the first
// ptk_comm_* call (dlopen; the copy torch already loaded is reused when present), so libptk itself has no
// link-time dependency on it and the single-GPU path never loads it.
//
// ptk_projector_bwd_allreduce overlaps the exchange with the projector backward: the flat grad buffer is
// [dW1 | db1 | dW2 | db2]; dW2 and db2 are computed first, so their all-reduce runs on the comm stream while
// the dA and dW1 GEMMs run on the compute stream; only the dW1 | db1 piece is exchanged after the last GEMM.
#include <dlfcn.h>
#include <stdio.h>
#include <string.h>

#include "../../include/ptk.h"
#include "ptk_internal.h"

using namespace ptk;

namespace {

// the subset of rccl.h used here (ABI of NCCL 2.x: ncclUniqueId is 128 bytes, enums are ints)
typedef struct { char internal[128]; } nccl_uid;
typedef void* nccl_comm;
enum { NCCL_FLOAT32 = 7 };
enum { NCCL_SUM = 0, NCCL_AVG = 4 };

struct Rccl {
  void* h = nullptr;
  int (*get_unique_id)(nccl_uid*) = nullptr;
  int (*comm_init_rank)(nccl_comm*, int, nccl_uid, int) = nullptr;
  int (*comm_destroy)(nccl_comm) = nullptr;
  int (*all_reduce)(const void*, void*, size_t, int, int, nccl_comm, hipStream_t) = nullptr;
  const char* (*error_string)(int) = nullptr;
};

Rccl* rccl() {
  static Rccl r;
  static bool tried = false;
  if (tried) return r.h ? &r : nullptr;
  tried = true;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);   // the process's RCCL (torch's), if loaded
  if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) return nullptr;
  r.get_unique_id = (int (*)(nccl_uid*))dlsym(h, "ncclGetUniqueId");
  r.comm_init_rank = (int (*)(nccl_comm*, int, nccl_uid, int))dlsym(h, "ncclCommInitRank");
  r.comm_destroy = (int (*)(nccl_comm))dlsym(h, "ncclCommDestroy");
  r.all_reduce = (int (*)(const void*, void*, size_t, int, int, nccl_comm, hipStream_t))dlsym(h, "ncclAllReduce");
  r.error_string = (const char* (*)(int))dlsym(h, "ncclGetErrorString");
  if (!r.get_unique_id || !r.comm_init_rank || !r.comm_destroy || !r.all_reduce || !r.error_string) return nullptr;
  r.h = h;
  return &r;
}

int rccl_error(const char* what, int rc) {
  Rccl* r = rccl();
  return set_error("%s: RCCL error %d (%s)", what, rc, r ? r->error_string(rc) : "?");
}

constexpr int COMM_EVENTS = 4;

}  // namespace

struct ptk_comm {
  nccl_comm c = nullptr;
  int world = 1, rank = 0, device = 0;
  hipEvent_t ev[COMM_EVENTS] = {};
};

extern "C" {

int ptk_comm_unique_id_bytes(void) { return (int)sizeof(nccl_uid); }

int ptk_comm_get_unique_id(void* out) {
  Rccl* r = rccl();
  if (!r) return set_error("ptk_comm: RCCL (librccl.so.1) not found");
  if (!out) return set_error("ptk_comm_get_unique_id: null output");
  nccl_uid id;
  const int rc = r->get_unique_id(&id);
  if (rc) return rccl_error("ncclGetUniqueId", rc);
  memcpy(out, &id, sizeof(id));
  return 0;
}

int ptk_comm_init(ptk_comm** out, const void* unique_id, int world, int rank) {
  if (!out || !unique_id) return set_error("ptk_comm_init: null argument");
  if (world < 1 || rank < 0 || rank >= world) return set_error("ptk_comm_init: rank %d of world %d", rank, world);
  Rccl* r = rccl();
  if (!r) return set_error("ptk_comm: RCCL (librccl.so.1) not found");
  ptk_comm* c = new ptk_comm;
  c->world = world;
  c->rank = rank;
  if (hipGetDevice(&c->device) != hipSuccess) { delete c; return set_error("ptk_comm_init: no HIP device"); }
  for (int i = 0; i < COMM_EVENTS; ++i)
    if (hipEventCreateWithFlags(&c->ev[i], hipEventDisableTiming) != hipSuccess) {
      for (int j = 0; j < i; ++j) (void)hipEventDestroy(c->ev[j]);
      delete c;
      return set_error("ptk_comm_init: hipEventCreate failed");
    }
  nccl_uid id;
  memcpy(&id, unique_id, sizeof(id));
  const int rc = r->comm_init_rank(&c->c, world, id, rank);
  if (rc) {
    for (int i = 0; i < COMM_EVENTS; ++i) (void)hipEventDestroy(c->ev[i]);
    delete c;
    return rccl_error("ncclCommInitRank", rc);
  }
  *out = c;
  return 0;
}

int ptk_comm_destroy(ptk_comm* c) {
  if (!c) return 0;
  Rccl* r = rccl();
  int rc = r && c->c ? r->comm_destroy(c->c) : 0;
  for (int i = 0; i < COMM_EVENTS; ++i) (void)hipEventDestroy(c->ev[i]);
  delete c;
  return rc ? rccl_error("ncclCommDestroy", rc) : 0;
}

int ptk_comm_world(const ptk_comm* c) { return c ? c->world : -1; }

static int allreduce(ptk_comm* c, float* buf, int64_t n, int op, hipStream_t st) {
  if (!c) return set_error("ptk_comm: null communicator");
  if (n <= 0) return 0;
  const int rc = rccl()->all_reduce(buf, buf, (size_t)n, NCCL_FLOAT32, op, c->c, st);
  return rc ? rccl_error("ncclAllReduce", rc) : 0;
}

int ptk_comm_allreduce_sum(ptk_comm* c, float* buf, int64_t n, void* stream) {
  return allreduce(c, buf, n, NCCL_SUM, (hipStream_t)stream);
}

int ptk_comm_allreduce_avg(ptk_comm* c, float* buf, int64_t n, void* stream) {
  return allreduce(c, buf, n, NCCL_AVG, (hipStream_t)stream);
}

int ptk_projector_bwd_allreduce(const ptk_projector* p, int rows, const void* x, const void* a, const void* h,
                                const void* dy, float* flat_grad, void* ws, size_t ws_bytes, ptk_comm* comm,
                                void* comm_stream, void* stream) {
  if (!comm) return set_error("ptk_projector_bwd_allreduce: null communicator");
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev != comm->device)
    return set_error("ptk_projector_bwd_allreduce: current device %d is not the communicator's device %d", dev,
                     comm->device);
  hipStream_t st = (hipStream_t)stream, cs = (hipStream_t)comm_stream;
  TailScratchScope tail(p->tail_ws, st);
  if (tail.status) return -1;
  StageScope stage("projector.bwd_allreduce", st);
  const long Dv = p->vision_dim, I = p->inter_dim, Dl = p->llm_dim;
  float* dw1 = flat_grad;
  float* db1 = dw1 + I * Dv;
  float* dw2 = db1 + I;
  float* db2 = dw2 + Dl * I;
  // the compute stream's earlier work (the grads' previous readers) precedes the comm stream's exchange
  if (hipEventRecord(comm->ev[0], st) != hipSuccess || hipStreamWaitEvent(cs, comm->ev[0], 0) != hipSuccess)
    return set_error("ptk_projector_bwd_allreduce: event");
  if (projector_bwd_stage(p, rows, x, a, h, dy, dw1, db1, dw2, db2, ws, ws_bytes, 0, st)) return -1;
  if (hipEventRecord(comm->ev[1], st) != hipSuccess || hipStreamWaitEvent(cs, comm->ev[1], 0) != hipSuccess)
    return set_error("ptk_projector_bwd_allreduce: event");
  if (allreduce(comm, dw2, Dl * I + Dl, NCCL_SUM, cs)) return -1;          // dW2 | db2 beside dA, dW1
  if (projector_bwd_stage(p, rows, x, a, h, dy, dw1, db1, dw2, db2, ws, ws_bytes, 1, st)) return -1;
  if (hipEventRecord(comm->ev[2], st) != hipSuccess || hipStreamWaitEvent(cs, comm->ev[2], 0) != hipSuccess)
    return set_error("ptk_projector_bwd_allreduce: event");
  if (allreduce(comm, dw1, I * Dv + I, NCCL_SUM, cs)) return -1;           // dW1 | db1
  if (hipEventRecord(comm->ev[3], cs) != hipSuccess || hipStreamWaitEvent(st, comm->ev[3], 0) != hipSuccess)
    return set_error("ptk_projector_bwd_allreduce: event");
  return 0;
}

}  // extern "C"

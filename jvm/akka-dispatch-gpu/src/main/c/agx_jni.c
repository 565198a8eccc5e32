/*
 * agx_jni.c — JNI glue for akka.dispatch.gpu.AgxJni (src/main/java/.../AgxJni.java): the C ABI of
 * include/akka_gpu.h for JDK 8 / 11 (the reference's CI JDKs, .travis.yml:10), where the Panama
 * binding (AgxNative.scala) is unavailable.  Each Java_* function forwards to one agx_* entry point;
 * a non-zero status becomes a Java exception with agx_last_error() as its message and the function
 * returns (JNI: the exception is raised when the native method returns).
 *
 * Build (where a JDK exists):
 *   cc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -I<repo>/include \
 *      agx_jni.c -L<repo>/akka_amd/lib -lakka_gpu -o libakka_gpu_jni.so
 * In this repository (no JDK in the image) __graft_entry__.build() compiles it against
 * tests/c/jni_min (a JNI-spec function table, test infrastructure only) and tests/c/jni_harness.c
 * drives every function through a fake JNIEnv on the GPU box.
 */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "akka_gpu.h"

#define ENG(h) ((agx_engine*)(intptr_t)(h))

/* status -> exception (AgxNative.check's mapping); returns 1 if one was raised */
static int raise(JNIEnv* env, agx_status st) {
  if (st == AGX_OK) return 0;
  const char* cls = st == AGX_EINVAL ? "akka/ConfigurationException" : "java/lang/IllegalStateException";
  char msg[640];
  if (st == AGX_EINVAL)
    snprintf(msg, sizeof msg, "akka-gpu: %s", agx_last_error());
  else if (st == AGX_ECAPACITY)
    snprintf(msg, sizeof msg, "akka-gpu: mailbox arena full: %s", agx_last_error());
  else
    snprintf(msg, sizeof msg, "akka-gpu status %d: %s", (int)st, agx_last_error());
  jclass c = (*env)->FindClass(env, cls);
  if (!c) c = (*env)->FindClass(env, "java/lang/RuntimeException");
  if (c) (*env)->ThrowNew(env, c, msg);
  return 1;
}

/* a Java int[] / long[] copied into malloc'd memory (NULL array -> NULL, *n = 0) */
static uint32_t* copy_ints(JNIEnv* env, jintArray a, jsize* n) {
  *n = a ? (*env)->GetArrayLength(env, a) : 0;
  if (!a) return NULL;
  uint32_t* p = (uint32_t*)malloc((size_t)(*n ? *n : 1) * 4);
  if (p && *n) (*env)->GetIntArrayRegion(env, a, 0, *n, (jint*)p);
  return p;
}
static uint64_t* copy_longs(JNIEnv* env, jlongArray a, jsize* n) {
  *n = a ? (*env)->GetArrayLength(env, a) : 0;
  if (!a) return NULL;
  uint64_t* p = (uint64_t*)malloc((size_t)(*n ? *n : 1) * 8);
  if (p && *n) (*env)->GetLongArrayRegion(env, a, 0, *n, (jlong*)p);
  return p;
}
static int oom(JNIEnv* env) {
  jclass c = (*env)->FindClass(env, "java/lang/OutOfMemoryError");
  if (c) (*env)->ThrowNew(env, c, "akka-gpu: host allocation failed");
  return 1;
}

JNIEXPORT jint JNICALL Java_akka_dispatch_gpu_AgxJni_abiVersion(JNIEnv* env, jclass k) {
  (void)env;
  (void)k;
  return (jint)agx_abi_version();
}

JNIEXPORT jstring JNICALL Java_akka_dispatch_gpu_AgxJni_lastError(JNIEnv* env, jclass k) {
  (void)k;
  return (*env)->NewStringUTF(env, agx_last_error());
}

JNIEXPORT jlong JNICALL Java_akka_dispatch_gpu_AgxJni_create(JNIEnv* env, jclass k, jint device, jlong n_actors,
                                                             jint throughput, jint capacity, jint n_words,
                                                             jint max_emit, jint n_ranks, jint rank, jint num_shards,
                                                             jint bucket_actors, jlong msg_capacity) {
  (void)k;
  agx_cfg c;
  memset(&c, 0, sizeof c);
  c.abi_version = AGX_ABI_VERSION;
  c.device = (uint32_t)device;
  c.n_actors = (uint64_t)n_actors;
  c.throughput = throughput < 0 ? 0u : (uint32_t)throughput; /* <= 0 behaves as 1 (Mailbox.scala:261) */
  c.capacity = (uint32_t)capacity;
  c.n_words = (uint32_t)n_words;
  c.max_emit = (uint32_t)max_emit;
  c.n_ranks = (uint32_t)n_ranks;
  c.rank = (uint32_t)rank;
  c.num_shards = (uint32_t)num_shards;
  c.bucket_actors = (uint32_t)bucket_actors;
  c.msg_capacity = (uint64_t)msg_capacity;
  agx_engine* e = NULL;
  if (raise(env, agx_create(&c, &e))) return 0;
  return (jlong)(intptr_t)e;
}

JNIEXPORT void JNICALL Java_akka_dispatch_gpu_AgxJni_destroy(JNIEnv* env, jclass k, jlong eng) {
  (void)k;
  raise(env, agx_destroy(ENG(eng)));
}

JNIEXPORT void JNICALL Java_akka_dispatch_gpu_AgxJni_registerRange(JNIEnv* env, jclass k, jlong eng, jlong first,
                                                                   jlong count, jint kind, jlongArray init,
                                                                   jint state_words) {
  (void)k;
  jsize n = 0;
  uint64_t* st = copy_longs(env, init, &n);
  if (init && !st) { oom(env); return; }
  if (st && (jlong)n < count * (jlong)state_words) {
    free(st);
    raise(env, AGX_EINVAL);
    return;
  }
  raise(env, agx_register_range(ENG(eng), (uint64_t)first, (uint64_t)count, (uint32_t)kind, st,
                                st ? (size_t)state_words * 8u : 0u));
  free(st);
}

JNIEXPORT void JNICALL Java_akka_dispatch_gpu_AgxJni_setMailboxClass(JNIEnv* env, jclass k, jlong eng, jint cls,
                                                                     jint capacity) {
  (void)k;
  raise(env, agx_set_mailbox_class(ENG(eng), (uint32_t)cls, (uint32_t)capacity));
}

JNIEXPORT void JNICALL Java_akka_dispatch_gpu_AgxJni_setMailbox(JNIEnv* env, jclass k, jlong eng, jlong first,
                                                                jlong count, jint cls) {
  (void)k;
  raise(env, agx_set_mailbox(ENG(eng), (uint64_t)first, (uint64_t)count, (uint32_t)cls));
}

JNIEXPORT void JNICALL Java_akka_dispatch_gpu_AgxJni_setRing(JNIEnv* env, jclass k, jlong eng, jint stride) {
  (void)k;
  raise(env, agx_set_ring(ENG(eng), (uint32_t)stride));
}

JNIEXPORT void JNICALL Java_akka_dispatch_gpu_AgxJni_setGossip(JNIEnv* env, jclass k, jlong eng, jint fanout,
                                                               jlong seed) {
  (void)k;
  raise(env, agx_set_gossip(ENG(eng), (uint32_t)fanout, (uint64_t)seed));
}

JNIEXPORT void JNICALL Java_akka_dispatch_gpu_AgxJni_setDeltaCrdt(JNIEnv* env, jclass k, jlong eng, jint max_delta) {
  (void)k;
  raise(env, agx_set_delta_crdt(ENG(eng), (uint32_t)max_delta));
}

JNIEXPORT void JNICALL Java_akka_dispatch_gpu_AgxJni_setBehaviors(JNIEnv* env, jclass k, jlong eng, jbyteArray cases,
                                                                  jint n_cases, jbyteArray acts, jint n_acts,
                                                                  jintArray first, jint n_beh) {
  (void)k;
  const jsize nc = cases ? (*env)->GetArrayLength(env, cases) : 0, na = acts ? (*env)->GetArrayLength(env, acts) : 0;
  if (n_cases < 0 || n_acts < 0 || (size_t)nc < (size_t)n_cases * sizeof(agx_case) ||
      (size_t)na < (size_t)n_acts * sizeof(agx_act)) {
    raise(env, AGX_EINVAL);
    return;
  }
  agx_case* c = (agx_case*)malloc((size_t)(n_cases ? n_cases : 1) * sizeof(agx_case));
  agx_act* a = (agx_act*)malloc((size_t)(n_acts ? n_acts : 1) * sizeof(agx_act));
  jsize nf = 0;
  uint32_t* f = copy_ints(env, first, &nf);
  if (!c || !a || (first && !f)) {
    free(c); free(a); free(f);
    oom(env);
    return;
  }
  if (n_cases) (*env)->GetByteArrayRegion(env, cases, 0, n_cases * (jsize)sizeof(agx_case), (jbyte*)c);
  if (n_acts) (*env)->GetByteArrayRegion(env, acts, 0, n_acts * (jsize)sizeof(agx_act), (jbyte*)a);
  if (!f || nf < n_beh + 1)
    raise(env, AGX_EINVAL);
  else
    raise(env, agx_set_behaviors(ENG(eng), c, (uint32_t)n_cases, a, (uint32_t)n_acts, f, (uint32_t)n_beh));
  free(c);
  free(a);
  free(f);
}

JNIEXPORT void JNICALL Java_akka_dispatch_gpu_AgxJni_setFanout(JNIEnv* env, jclass k, jlong eng, jint kk, jlong seed,
                                                               jintArray cdf, jintArray perm) {
  (void)k;
  jsize n1 = 0, n2 = 0;
  uint32_t* c = copy_ints(env, cdf, &n1);
  uint32_t* p = copy_ints(env, perm, &n2);
  if (!c || !p || n1 != n2)
    raise(env, AGX_EINVAL);
  else
    raise(env, agx_set_fanout(ENG(eng), (uint32_t)kk, (uint64_t)seed, c, p, (uint64_t)n1));
  free(c);
  free(p);
}

JNIEXPORT void JNICALL Java_akka_dispatch_gpu_AgxJni_setGraph(JNIEnv* env, jclass k, jlong eng, jlongArray row_ptr,
                                                              jintArray col) {
  (void)k;
  uint64_t n_actors = 0;
  if (raise(env, agx_get_shape(ENG(eng), &n_actors, NULL))) return;
  jsize nr = 0, nc = 0;
  uint64_t* r = copy_longs(env, row_ptr, &nr);
  uint32_t* c = copy_ints(env, col, &nc);
  /* agx_set_graph reads row_ptr[0 .. n_actors] and col[0 .. row_ptr[n_actors]) once row_ptr is
   * monotone (it checks that before reading col; checked here too, so an over-long row cannot
   * reach the native copy of col) */
  int mono = r != NULL && (uint64_t)nr == n_actors + 1;
  for (uint64_t i = 0; mono && i < n_actors; ++i) mono = r[i] <= r[i + 1];
  if (!mono || (uint64_t)nc < r[n_actors] || (r[n_actors] && !c))
    raise(env, AGX_EINVAL);
  else
    raise(env, agx_set_graph(ENG(eng), r, c ? c : (const uint32_t*)r));
  free(r);
  free(c);
}

/* agx_tell: no array, no lock -- one call per ActorRef.! (GpuEngine.tell) */
JNIEXPORT jboolean JNICALL Java_akka_dispatch_gpu_AgxJni_tell(JNIEnv* env, jclass k, jlong eng, jint dst, jint src,
                                                             jint pay) {
  (void)k;
  int32_t sched = 0;
  raise(env, agx_tell(ENG(eng), (uint32_t)dst, (uint32_t)src, (uint32_t)pay, &sched));
  return sched ? JNI_TRUE : JNI_FALSE;
}

JNIEXPORT jboolean JNICALL Java_akka_dispatch_gpu_AgxJni_pumpIdle(JNIEnv* env, jclass k, jlong eng) {
  (void)k;
  int32_t again = 0;
  raise(env, agx_pump_idle(ENG(eng), &again));
  return again ? JNI_TRUE : JNI_FALSE;
}

/* agx_pump_cancel: the executor rejected the pump -- back to idle, no re-check */
JNIEXPORT void JNICALL Java_akka_dispatch_gpu_AgxJni_pumpCancel(JNIEnv* env, jclass k, jlong eng) {
  (void)k;
  raise(env, agx_pump_cancel(ENG(eng)));
}

JNIEXPORT void JNICALL Java_akka_dispatch_gpu_AgxJni_stageTells(JNIEnv* env, jclass k, jlong eng, jobject dst,
                                                                jobject src, jobject pay, jint n) {
  (void)k;
  const uint32_t* d = dst ? (const uint32_t*)(*env)->GetDirectBufferAddress(env, dst) : NULL;
  const uint32_t* s = src ? (const uint32_t*)(*env)->GetDirectBufferAddress(env, src) : NULL;
  const uint32_t* p = pay ? (const uint32_t*)(*env)->GetDirectBufferAddress(env, pay) : NULL;
  const jlong need = (jlong)n * 4;
  if (n < 0 || !d || !p || (src && !s) || (*env)->GetDirectBufferCapacity(env, dst) < need ||
      (*env)->GetDirectBufferCapacity(env, pay) < need || (src && (*env)->GetDirectBufferCapacity(env, src) < need)) {
    raise(env, AGX_EINVAL);
    return;
  }
  raise(env, agx_stage_tells(ENG(eng), d, s, p, (size_t)n));
}

JNIEXPORT void JNICALL Java_akka_dispatch_gpu_AgxJni_stageTellsArrays(JNIEnv* env, jclass k, jlong eng, jintArray dst,
                                                                      jintArray src, jintArray pay, jint n) {
  (void)k;
  jsize nd = 0, ns = 0, np = 0;
  uint32_t* d = copy_ints(env, dst, &nd);
  uint32_t* s = copy_ints(env, src, &ns);
  uint32_t* p = copy_ints(env, pay, &np);
  if (n < 0 || !d || !p || nd < n || np < n || (src && ns < n))
    raise(env, AGX_EINVAL);
  else
    raise(env, agx_stage_tells(ENG(eng), d, s, p, (size_t)n));
  free(d);
  free(s);
  free(p);
}

static void put_stats(JNIEnv* env, jlongArray out, const agx_stats* st) {
  const jlong v[8] = {(jlong)st->delivered, (jlong)st->dead_letters, (jlong)st->unhandled, (jlong)st->emitted,
                      (jlong)st->staged,    (jlong)st->supersteps,   (jlong)st->in_flight, (jlong)st->bytes_alg};
  const jsize n = (*env)->GetArrayLength(env, out);
  (*env)->SetLongArrayRegion(env, out, 0, n < 8 ? n : 8, v);
}

JNIEXPORT void JNICALL Java_akka_dispatch_gpu_AgxJni_run(JNIEnv* env, jclass k, jlong eng, jint max_steps,
                                                         jlongArray stats) {
  (void)k;
  agx_stats st;
  memset(&st, 0, sizeof st);
  if (raise(env, agx_run(ENG(eng), (uint32_t)max_steps, stats ? &st : NULL))) return;
  if (stats) put_stats(env, stats, &st);
}

JNIEXPORT void JNICALL Java_akka_dispatch_gpu_AgxJni_getStats(JNIEnv* env, jclass k, jlong eng, jlongArray stats) {
  (void)k;
  agx_stats st;
  memset(&st, 0, sizeof st);
  if (raise(env, agx_get_stats(ENG(eng), &st))) return;
  if (stats) put_stats(env, stats, &st);
}

JNIEXPORT void JNICALL Java_akka_dispatch_gpu_AgxJni_readState(JNIEnv* env, jclass k, jlong eng, jlong first,
                                                               jlong count, jlongArray words, jbyteArray alive) {
  (void)k;
  uint32_t n_words = 0;
  if (raise(env, agx_get_shape(ENG(eng), NULL, &n_words))) return;
  const jsize nw = words ? (*env)->GetArrayLength(env, words) : 0;
  const jsize na = alive ? (*env)->GetArrayLength(env, alive) : 0;
  /* agx_read_state writes count x n_words u64: the array must hold exactly that */
  if (count < 0 || count > 0x7FFFFFFFll || (alive && na < count) ||
      (words && (jlong)nw != count * (jlong)n_words)) {
    raise(env, AGX_EINVAL);
    return;
  }
  uint64_t* w = words ? (uint64_t*)malloc((size_t)(nw ? nw : 1) * 8) : NULL;
  uint8_t* a = alive ? (uint8_t*)malloc((size_t)(na ? na : 1)) : NULL;
  if ((words && !w) || (alive && !a)) {
    free(w); free(a);
    oom(env);
    return;
  }
  if (!raise(env, agx_read_state(ENG(eng), (uint64_t)first, (uint64_t)count, w, a))) {
    if (w && nw) (*env)->SetLongArrayRegion(env, words, 0, nw, (const jlong*)w);
    if (a && count) (*env)->SetByteArrayRegion(env, alive, 0, (jsize)count, (const jbyte*)a);
  }
  free(w);
  free(a);
}

JNIEXPORT void JNICALL Java_akka_dispatch_gpu_AgxJni_setOutbound(JNIEnv* env, jclass k, jlong eng, jint first_host,
                                                                 jint n_host, jlong capacity) {
  (void)k;
  raise(env, agx_set_outbound(ENG(eng), (uint32_t)first_host, (uint32_t)n_host, (uint64_t)capacity));
}

JNIEXPORT jint JNICALL Java_akka_dispatch_gpu_AgxJni_takeOutbound(JNIEnv* env, jclass k, jlong eng, jintArray dst,
                                                                  jintArray src, jintArray pay, jint cap) {
  (void)k;
  if (cap < 0 || !dst || !src || !pay || (*env)->GetArrayLength(env, dst) < cap ||
      (*env)->GetArrayLength(env, src) < cap || (*env)->GetArrayLength(env, pay) < cap) {
    raise(env, AGX_EINVAL);
    return 0;
  }
  uint32_t* d = (uint32_t*)malloc((size_t)(cap ? cap : 1) * 4);
  uint32_t* s = (uint32_t*)malloc((size_t)(cap ? cap : 1) * 4);
  uint32_t* p = (uint32_t*)malloc((size_t)(cap ? cap : 1) * 4);
  uint64_t n = 0;
  if (!d || !s || !p) {
    free(d); free(s); free(p);
    oom(env);
    return 0;
  }
  if (!raise(env, agx_take_outbound(ENG(eng), d, s, p, (uint64_t)cap, &n)) && n) {
    (*env)->SetIntArrayRegion(env, dst, 0, (jsize)n, (const jint*)d);
    (*env)->SetIntArrayRegion(env, src, 0, (jsize)n, (const jint*)s);
    (*env)->SetIntArrayRegion(env, pay, 0, (jsize)n, (const jint*)p);
  }
  free(d);
  free(s);
  free(p);
  return (jint)n;
}

JNIEXPORT jint JNICALL Java_akka_dispatch_gpu_AgxJni_shardId(JNIEnv* env, jclass k, jint id, jint num_shards) {
  (void)env;
  (void)k;
  return (jint)agx_shard_id((uint32_t)id, (uint32_t)num_shards);
}

JNIEXPORT jint JNICALL Java_akka_dispatch_gpu_AgxJni_owner(JNIEnv* env, jclass k, jint id, jint num_shards,
                                                           jint n_ranks) {
  (void)env;
  (void)k;
  return (jint)agx_owner((uint32_t)id, (uint32_t)num_shards, (uint32_t)n_ranks);
}

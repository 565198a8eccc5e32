/*
 * jni_harness.c -- drives the JNI glue (jvm/akka-dispatch-gpu/src/main/c/agx_jni.c, built into
 * akka_amd/lib/libakka_gpu_jni.so) through a fake JNIEnv, in the order the JDK 8/11 shim calls it,
 * against the real libakka_gpu.so on the GPU.  The fake env implements the JNI functions the glue
 * uses (FindClass, ThrowNew, NewStringUTF, Get/SetXxxArrayRegion, GetArrayLength,
 * GetDirectBufferAddress / Capacity) over plain C arrays; a ThrowNew is recorded as the pending
 * exception, as a JVM would raise it when the native method returns.
 *
 * Checks, each citing the reference behaviour it mirrors:
 *   - configuration errors surface as akka.ConfigurationException (Dispatchers.scala:248-260:
 *     a bad dispatcher/mailbox config is a ConfigurationException), capacity errors as
 *     IllegalStateException, never as a crash;
 *   - ActorModelSpec "handle queueing from multiple threads" (ActorModelSpec.scala:323-336):
 *     messages received by dispatch == messages processed by the actor;
 *   - per-actor mailboxes (Mailboxes.scala:204-260, bounded-capacity:N): a BoundedMailbox(10)
 *     actor beside unbounded ones drops exactly the messages beyond 10 (MailboxConfigSpec:47-66);
 *   - sender() ! reply to a JVM actor (ActorCell.scala:583-587): a GPU PingPong actor answering a
 *     JVM probe -- the replies leave the engine through the outbox in per-sender order and the
 *     probe answers them, until the GPU actor stops (BenchmarkActors.PingPong);
 *   - the lock-free tell path (AgxJni.tell / pumpIdle -> agx_tell / agx_pump_idle): a burst of
 *     tells to an idle engine submits ONE pump (Mailbox.setAsScheduled, Mailbox.scala:185-194), and
 *     tells from 4 threads racing a pump that resubmits itself only when pumpIdle says so are all
 *     delivered (ActorModelSpec "handle queueing from multiple threads", :323-336) -- 100000 of them,
 *     6x the engine's message capacity: an unbounded mailbox never refuses an enqueue
 *     (AbstractNodeQueue.java:79-82), so the tells that do not fit wait for a later pump;
 *   - a pump budget (gpu.supersteps-per-pump) that stops with mail in flight: pumpIdle asks for
 *     another run until the mail is delivered (Mailbox.run re-registers while hasMessages,
 *     Mailbox.scala:227-240); pumpCancel (the executor rejected the pump) returns the engine to
 *     idle so the next tell submits again (Dispatcher.scala:130-138).
 * Exit 0 = every check passed.  Run by tests/test_abi_c.py on the GPU box.
 */
#include <pthread.h>
#include <stdatomic.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "jni.h" /* tests/c/jni_min */
#include "../../include/akka_gpu.h"

/* ------------------------------------------------------------------ the glue's entry points */
jint Java_akka_dispatch_gpu_AgxJni_abiVersion(JNIEnv*, jclass);
jstring Java_akka_dispatch_gpu_AgxJni_lastError(JNIEnv*, jclass);
jlong Java_akka_dispatch_gpu_AgxJni_create(JNIEnv*, jclass, jint, jlong, jint, jint, jint, jint, jint, jint, jint, jint,
                                           jlong);
void Java_akka_dispatch_gpu_AgxJni_destroy(JNIEnv*, jclass, jlong);
void Java_akka_dispatch_gpu_AgxJni_registerRange(JNIEnv*, jclass, jlong, jlong, jlong, jint, jlongArray, jint);
void Java_akka_dispatch_gpu_AgxJni_setMailboxClass(JNIEnv*, jclass, jlong, jint, jint);
void Java_akka_dispatch_gpu_AgxJni_setMailbox(JNIEnv*, jclass, jlong, jlong, jlong, jint);
void Java_akka_dispatch_gpu_AgxJni_setRing(JNIEnv*, jclass, jlong, jint);
void Java_akka_dispatch_gpu_AgxJni_stageTells(JNIEnv*, jclass, jlong, jobject, jobject, jobject, jint);
void Java_akka_dispatch_gpu_AgxJni_stageTellsArrays(JNIEnv*, jclass, jlong, jintArray, jintArray, jintArray, jint);
void Java_akka_dispatch_gpu_AgxJni_run(JNIEnv*, jclass, jlong, jint, jlongArray);
jboolean Java_akka_dispatch_gpu_AgxJni_tell(JNIEnv*, jclass, jlong, jint, jint, jint);
jboolean Java_akka_dispatch_gpu_AgxJni_pumpIdle(JNIEnv*, jclass, jlong);
void Java_akka_dispatch_gpu_AgxJni_pumpCancel(JNIEnv*, jclass, jlong);
void Java_akka_dispatch_gpu_AgxJni_getStats(JNIEnv*, jclass, jlong, jlongArray);
void Java_akka_dispatch_gpu_AgxJni_readState(JNIEnv*, jclass, jlong, jlong, jlong, jlongArray, jbyteArray);
void Java_akka_dispatch_gpu_AgxJni_setGraph(JNIEnv*, jclass, jlong, jlongArray, jintArray);
void Java_akka_dispatch_gpu_AgxJni_setOutbound(JNIEnv*, jclass, jlong, jint, jint, jlong);
jint Java_akka_dispatch_gpu_AgxJni_takeOutbound(JNIEnv*, jclass, jlong, jintArray, jintArray, jintArray, jint);
jint Java_akka_dispatch_gpu_AgxJni_shardId(JNIEnv*, jclass, jint, jint);

/* the typed slots sit at their JNI-specification indices */
#define SLOT(f) (offsetof(struct JNINativeInterface_, f) / sizeof(void*))
_Static_assert(SLOT(FindClass) == 6, "FindClass");
_Static_assert(SLOT(ThrowNew) == 14, "ThrowNew");
_Static_assert(SLOT(NewStringUTF) == 167, "NewStringUTF");
_Static_assert(SLOT(GetArrayLength) == 171, "GetArrayLength");
_Static_assert(SLOT(GetByteArrayRegion) == 200, "GetByteArrayRegion");
_Static_assert(SLOT(GetIntArrayRegion) == 203, "GetIntArrayRegion");
_Static_assert(SLOT(GetLongArrayRegion) == 204, "GetLongArrayRegion");
_Static_assert(SLOT(SetByteArrayRegion) == 208, "SetByteArrayRegion");
_Static_assert(SLOT(SetIntArrayRegion) == 211, "SetIntArrayRegion");
_Static_assert(SLOT(SetLongArrayRegion) == 212, "SetLongArrayRegion");
_Static_assert(SLOT(GetDirectBufferAddress) == 230, "GetDirectBufferAddress");
_Static_assert(SLOT(GetDirectBufferCapacity) == 231, "GetDirectBufferCapacity");

/* ------------------------------------------------------------------ the fake JVM */
enum { T_CLASS, T_STRING, T_ARRAY, T_DIRECT };
struct _jobject {
  int type;
  size_t elem;  /* array element size */
  jsize len;    /* elements (arrays), bytes (direct buffers) */
  void* data;
  char name[128];
};

static char pending_cls[128], pending_msg[1024];
static int failures = 0, n_exceptions = 0;

static jobject new_obj(int type, size_t elem, jsize len) {
  jobject o = (jobject)calloc(1, sizeof(struct _jobject));
  o->type = type;
  o->elem = elem;
  o->len = len;
  o->data = calloc((size_t)(len ? len : 1), elem ? elem : 1);
  return o;
}
static void free_obj(jobject o) {
  if (!o) return;
  free(o->data);
  free(o);
}
static jclass f_FindClass(JNIEnv* env, const char* name) {
  (void)env;
  jobject c = new_obj(T_CLASS, 1, 0);
  snprintf(c->name, sizeof c->name, "%s", name);
  return c; /* (a local reference: leaked until the harness exits) */
}
static jint f_ThrowNew(JNIEnv* env, jclass c, const char* msg) {
  (void)env;
  snprintf(pending_cls, sizeof pending_cls, "%s", c->name);
  snprintf(pending_msg, sizeof pending_msg, "%s", msg);
  ++n_exceptions;
  return JNI_OK;
}
static jstring f_NewStringUTF(JNIEnv* env, const char* s) {
  (void)env;
  jobject o = new_obj(T_STRING, 1, (jsize)strlen(s) + 1);
  memcpy(o->data, s, strlen(s) + 1);
  return o;
}
static jsize f_GetArrayLength(JNIEnv* env, jarray a) {
  (void)env;
  return a->len;
}
static void region_get(jarray a, jsize s, jsize n, void* out, size_t elem) {
  if (a->type != T_ARRAY || a->elem != elem || s < 0 || n < 0 || s + n > a->len) {
    fprintf(stderr, "FAIL: bad array region read\n");
    ++failures;
    return;
  }
  memcpy(out, (char*)a->data + (size_t)s * elem, (size_t)n * elem);
}
static void region_set(jarray a, jsize s, jsize n, const void* in, size_t elem) {
  if (a->type != T_ARRAY || a->elem != elem || s < 0 || n < 0 || s + n > a->len) {
    fprintf(stderr, "FAIL: bad array region write\n");
    ++failures;
    return;
  }
  memcpy((char*)a->data + (size_t)s * elem, in, (size_t)n * elem);
}
static void f_GetByteArrayRegion(JNIEnv* e, jbyteArray a, jsize s, jsize n, jbyte* o) { (void)e; region_get(a, s, n, o, 1); }
static void f_GetIntArrayRegion(JNIEnv* e, jintArray a, jsize s, jsize n, jint* o) { (void)e; region_get(a, s, n, o, 4); }
static void f_GetLongArrayRegion(JNIEnv* e, jlongArray a, jsize s, jsize n, jlong* o) { (void)e; region_get(a, s, n, o, 8); }
static void f_SetByteArrayRegion(JNIEnv* e, jbyteArray a, jsize s, jsize n, const jbyte* i) { (void)e; region_set(a, s, n, i, 1); }
static void f_SetIntArrayRegion(JNIEnv* e, jintArray a, jsize s, jsize n, const jint* i) { (void)e; region_set(a, s, n, i, 4); }
static void f_SetLongArrayRegion(JNIEnv* e, jlongArray a, jsize s, jsize n, const jlong* i) { (void)e; region_set(a, s, n, i, 8); }
static void* f_GetDirectBufferAddress(JNIEnv* e, jobject b) {
  (void)e;
  return b && b->type == T_DIRECT ? b->data : NULL;
}
static jlong f_GetDirectBufferCapacity(JNIEnv* e, jobject b) {
  (void)e;
  return b && b->type == T_DIRECT ? b->len : -1;
}

static struct JNINativeInterface_ table;
static JNIEnv env_v = &table;
static JNIEnv* const env = &env_v;

#define CHECK(cond, ...)                                    \
  do {                                                      \
    if (!(cond)) {                                          \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);  \
      fprintf(stderr, __VA_ARGS__);                         \
      fprintf(stderr, " (pending %s: %s)\n", pending_cls, pending_msg); \
      ++failures;                                           \
    }                                                       \
  } while (0)
/* a native call that must not raise */
#define NOEXC(call)                                                     \
  do {                                                                  \
    const int _n0 = n_exceptions;                                       \
    call;                                                               \
    CHECK(n_exceptions == _n0, "%s raised %s", #call, pending_cls);     \
  } while (0)
/* a native call that must raise `cls` */
#define RAISES(cls, call)                                                                \
  do {                                                                                   \
    const int _n0 = n_exceptions;                                                        \
    call;                                                                                \
    CHECK(n_exceptions == _n0 + 1 && strcmp(pending_cls, cls) == 0, "%s should raise %s", #call, cls); \
  } while (0)

static jintArray ints(jsize n) { return new_obj(T_ARRAY, 4, n); }
static jlongArray longs(jsize n) { return new_obj(T_ARRAY, 8, n); }
static jbyteArray bytes(jsize n) { return new_obj(T_ARRAY, 1, n); }
static jobject direct_ints(jsize n) { return new_obj(T_DIRECT, 1, n * 4); }
#define I(a) ((jint*)(a)->data)
#define L(a) ((jlong*)(a)->data)
#define B(a) ((jbyte*)(a)->data)

/* a sender thread of the lock-free tell path: TELLS tells to COUNTER actor 3100 + t, payloads 1..TELLS;
   a tell that answers "submit" counts one pump submission */
enum { TELLS = 25000 }; /* 4 x 25000 = 100000 tells: 6x the engine's msg_capacity (MSGCAP below) -- the
                          pump takes what fits, the rest wait in the queue (back-pressure, never loss) */
enum { MSGCAP = 16384 };
typedef struct { jlong eng; int t; } tell_arg;
static atomic_long t_submitted;
static atomic_int ta_done[4];
static void* teller(void* p) {
  const tell_arg* a = (const tell_arg*)p;
  for (jint i = 1; i <= TELLS; ++i)
    if (Java_akka_dispatch_gpu_AgxJni_tell(env, NULL, a->eng, 3100 + a->t, AGX_NO_SENDER, i)) atomic_fetch_add(&t_submitted, 1);
  atomic_store(&ta_done[a->t], 1);
  return NULL;
}

int main(void) {
  table.FindClass = f_FindClass;
  table.ThrowNew = f_ThrowNew;
  table.NewStringUTF = f_NewStringUTF;
  table.GetArrayLength = f_GetArrayLength;
  table.GetByteArrayRegion = f_GetByteArrayRegion;
  table.GetIntArrayRegion = f_GetIntArrayRegion;
  table.GetLongArrayRegion = f_GetLongArrayRegion;
  table.SetByteArrayRegion = f_SetByteArrayRegion;
  table.SetIntArrayRegion = f_SetIntArrayRegion;
  table.SetLongArrayRegion = f_SetLongArrayRegion;
  table.GetDirectBufferAddress = f_GetDirectBufferAddress;
  table.GetDirectBufferCapacity = f_GetDirectBufferCapacity;
  const jclass K = NULL;

  CHECK(Java_akka_dispatch_gpu_AgxJni_abiVersion(env, K) == (jint)AGX_ABI_VERSION, "abi version");
  CHECK(Java_akka_dispatch_gpu_AgxJni_shardId(env, K, 42, 1000) == 662, "shard of 42");

  /* configuration errors -> ConfigurationException, handle 0 */
  jlong bad = 0;
  RAISES("akka/ConfigurationException", bad = Java_akka_dispatch_gpu_AgxJni_create(env, K, 0, 0, 5, 0, 2, 1, 1, 0, 1000, 0, 0));
  CHECK(bad == 0, "no handle for a bad config");
  RAISES("akka/ConfigurationException", Java_akka_dispatch_gpu_AgxJni_create(env, K, 0, 4096, 5, 0, 2, 1, 1, 0, 1000, 48, 0));

  enum { N = 4096, HOST = N, NHOST = 16, PROBE = HOST + 3 };
  jlong eng = 0;
  NOEXC(eng = Java_akka_dispatch_gpu_AgxJni_create(env, K, 0, N, 5, 0, 2, 1, 1, 0, 1000, 0, MSGCAP));
  CHECK(eng != 0, "engine handle");
  /* actorOf: COUNTER actors; a PingPong actor at 200 with 5 messages left (BenchmarkActors.PingPong) */
  NOEXC(Java_akka_dispatch_gpu_AgxJni_registerRange(env, K, eng, 0, N, AGX_KIND_COUNTER, NULL, 2));
  jlongArray pp = longs(2);
  L(pp)[0] = 5;
  NOEXC(Java_akka_dispatch_gpu_AgxJni_registerRange(env, K, eng, 200, 1, AGX_KIND_PINGPONG, pp, 2));
  RAISES("akka/ConfigurationException", Java_akka_dispatch_gpu_AgxJni_registerRange(env, K, eng, 0, 1, 99, NULL, 2));
  /* mailbox-type bounded-capacity:10 for actors 100..107 only (Mailboxes.lookupConfigurator) */
  NOEXC(Java_akka_dispatch_gpu_AgxJni_setMailboxClass(env, K, eng, 1, 10));
  NOEXC(Java_akka_dispatch_gpu_AgxJni_setMailbox(env, K, eng, 100, 8, 1));
  RAISES("akka/ConfigurationException", Java_akka_dispatch_gpu_AgxJni_setMailbox(env, K, eng, 0, 1, 99));
  /* JVM actors (TestProbes) get ids [N, N + 16): GPU tells to them leave through the outbox */
  NOEXC(Java_akka_dispatch_gpu_AgxJni_setOutbound(env, K, eng, HOST, NHOST, 1 << 16));

  /* ActorModelSpec: 200 "threads" x 50 messages to COUNTER actor 3 through a direct buffer,
     20 messages to the bounded actor 101, 20 to the unbounded actor 120 */
  const jint nt = 200 * 50 + 40;
  jobject d = direct_ints(nt), s = direct_ints(nt), p = direct_ints(nt);
  uint32_t* dd = (uint32_t*)d->data;
  uint32_t* sd = (uint32_t*)s->data;
  uint32_t* pd = (uint32_t*)p->data;
  for (jint i = 0; i < 200 * 50; ++i) {
    dd[i] = 3;
    sd[i] = AGX_NO_SENDER;
    pd[i] = (uint32_t)i;
  }
  for (jint i = 0; i < 20; ++i) {
    dd[200 * 50 + i] = 101;
    dd[200 * 50 + 20 + i] = 120;
    sd[200 * 50 + i] = sd[200 * 50 + 20 + i] = PROBE;
    pd[200 * 50 + i] = pd[200 * 50 + 20 + i] = (uint32_t)i + 1;
  }
  NOEXC(Java_akka_dispatch_gpu_AgxJni_stageTells(env, K, eng, d, s, p, nt));
  RAISES("akka/ConfigurationException", Java_akka_dispatch_gpu_AgxJni_stageTells(env, K, eng, d, s, p, nt + 1));
  jlongArray st = longs(8);
  NOEXC(Java_akka_dispatch_gpu_AgxJni_run(env, K, eng, 1 << 30, st));
  CHECK(L(st)[0] == 200 * 50 + 10 + 20, "delivered %lld", (long long)L(st)[0]);
  CHECK(L(st)[1] == 10, "dead letters %lld (bounded-capacity:10 drops 10 of 20)", (long long)L(st)[1]);
  CHECK(L(st)[6] == 0, "in flight");
  jlongArray w = longs(2); /* count 1 x n_words 2 */
  jbyteArray al = bytes(3);
  /* arrays that do not match count x n_words: rejected before any native write */
  jlongArray wshort = longs(1), wlong = longs(3);
  RAISES("akka/ConfigurationException", Java_akka_dispatch_gpu_AgxJni_readState(env, K, eng, 3, 1, wshort, al));
  RAISES("akka/ConfigurationException", Java_akka_dispatch_gpu_AgxJni_readState(env, K, eng, 3, 1, wlong, al));
  RAISES("akka/ConfigurationException", Java_akka_dispatch_gpu_AgxJni_readState(env, K, eng, 0, 2, w, al));
  /* a CSR whose rowPtr is shorter than n_actors + 1 (or col shorter than rowPtr[n]): rejected */
  jlongArray rp_short = longs(3);
  jintArray col1 = ints(1);
  RAISES("akka/ConfigurationException", Java_akka_dispatch_gpu_AgxJni_setGraph(env, K, eng, rp_short, col1));
  jlongArray rp = longs(N + 1);
  for (jint i = 0; i <= N; ++i) L(rp)[i] = i < 8 ? i : 8; /* actors 0..7 have one edge each */
  RAISES("akka/ConfigurationException", Java_akka_dispatch_gpu_AgxJni_setGraph(env, K, eng, rp, col1));
  /* a non-monotone rowPtr whose last entry fits col ([0, 100, 1, 1, ...]): rejected before the
   * native copy of col is read */
  for (jint i = 0; i <= N; ++i) L(rp)[i] = i == 1 ? 100 : i == 0 ? 0 : 1;
  RAISES("akka/ConfigurationException", Java_akka_dispatch_gpu_AgxJni_setGraph(env, K, eng, rp, col1));
  free_obj(wshort);
  free_obj(wlong);
  free_obj(rp_short);
  free_obj(rp);
  free_obj(col1);
  NOEXC(Java_akka_dispatch_gpu_AgxJni_readState(env, K, eng, 3, 1, w, al));
  CHECK(L(w)[0] == 200 * 50 && B(al)[0] == 1, "msgsProcessed == msgsReceived (%lld)", (long long)L(w)[0]);
  NOEXC(Java_akka_dispatch_gpu_AgxJni_readState(env, K, eng, 101, 1, w, al));
  CHECK(L(w)[0] == 10 && L(w)[1] == 55, "bounded actor kept the first 10 (FIFO): count %lld sum %lld",
        (long long)L(w)[0], (long long)L(w)[1]);
  NOEXC(Java_akka_dispatch_gpu_AgxJni_readState(env, K, eng, 120, 1, w, al));
  CHECK(L(w)[0] == 20 && L(w)[1] == 210, "unbounded neighbour kept all 20");

  /* sender() ! reply: the probe pings PingPong actor 200; every reply comes back through the outbox
     and the probe answers it, until the actor stops after 6 messages (left 5 -> 0) */
  jintArray od = ints(64), os = ints(64), op = ints(64), td = ints(1), ts = ints(1), tp = ints(1);
  I(td)[0] = 200;
  I(ts)[0] = PROBE;
  I(tp)[0] = 7;
  int replies = 0;
  for (int round = 0; round < 10; ++round) {
    NOEXC(Java_akka_dispatch_gpu_AgxJni_stageTellsArrays(env, K, eng, td, ts, tp, 1));
    NOEXC(Java_akka_dispatch_gpu_AgxJni_run(env, K, eng, 1 << 30, st));
    jint n = -1;
    NOEXC(n = Java_akka_dispatch_gpu_AgxJni_takeOutbound(env, K, eng, od, os, op, 64));
    if (n == 0) break;
    CHECK(n == 1 && I(od)[0] == PROBE && I(os)[0] == 200 && I(op)[0] == 7 + round, "reply %d: n=%d dst=%d src=%d pay=%d",
          round, n, I(od)[0], I(os)[0], I(op)[0]);
    ++replies;
    I(tp)[0] = I(op)[0] + 1; /* the probe answers the reply */
  }
  CHECK(replies == 6, "PingPong replied %d times (6 = left + 1)", replies);
  NOEXC(Java_akka_dispatch_gpu_AgxJni_readState(env, K, eng, 200, 1, w, al));
  CHECK(L(w)[1] == 6 && B(al)[0] == 0, "PingPong processed 6 and stopped");
  NOEXC(Java_akka_dispatch_gpu_AgxJni_getStats(env, K, eng, st));
  CHECK(L(st)[1] == 10 + 1, "the 7th ping is a dead letter (actor stopped)");

  /* several replies from several GPU actors: per-sender order survives the outbox */
  for (int a = 0; a < 8; ++a) {
    L(pp)[0] = 100;
    NOEXC(Java_akka_dispatch_gpu_AgxJni_registerRange(env, K, eng, 300 + a, 1, AGX_KIND_PINGPONG, pp, 2));
  }
  jintArray md = ints(8 * 5), ms = ints(8 * 5), mp = ints(8 * 5);
  for (int a = 0; a < 8; ++a)
    for (int k = 0; k < 5; ++k) {
      I(md)[a * 5 + k] = 300 + a;
      I(ms)[a * 5 + k] = HOST + (a % 4);
      I(mp)[a * 5 + k] = 1000 * a + k;
    }
  NOEXC(Java_akka_dispatch_gpu_AgxJni_stageTellsArrays(env, K, eng, md, ms, mp, 40));
  NOEXC(Java_akka_dispatch_gpu_AgxJni_run(env, K, eng, 1 << 30, st));
  jint n = 0;
  NOEXC(n = Java_akka_dispatch_gpu_AgxJni_takeOutbound(env, K, eng, od, os, op, 64));
  CHECK(n == 40, "40 replies (%d)", n);
  int next[8] = {0};
  for (jint i = 0; i < n; ++i) {
    const int a = I(os)[i] - 300;
    CHECK(a >= 0 && a < 8 && I(od)[i] == HOST + (a % 4) && I(op)[i] == 1000 * a + next[a], "reply order of actor %d", a);
    if (a >= 0 && a < 8) ++next[a];
  }
  NOEXC(n = Java_akka_dispatch_gpu_AgxJni_takeOutbound(env, K, eng, od, os, op, 64));
  CHECK(n == 0, "outbox drained");

  /* an outbox overflow is reported once by takeOutbound (IllegalStateException) and the engine
     stays usable: the kept replies come out of the next take, later runs work */
  NOEXC(Java_akka_dispatch_gpu_AgxJni_setOutbound(env, K, eng, HOST, NHOST, 4));
  NOEXC(Java_akka_dispatch_gpu_AgxJni_stageTellsArrays(env, K, eng, md, ms, mp, 40));
  NOEXC(Java_akka_dispatch_gpu_AgxJni_run(env, K, eng, 1 << 30, st));
  RAISES("java/lang/IllegalStateException", Java_akka_dispatch_gpu_AgxJni_takeOutbound(env, K, eng, od, os, op, 64));
  NOEXC(n = Java_akka_dispatch_gpu_AgxJni_takeOutbound(env, K, eng, od, os, op, 64));
  CHECK(n == 4, "the 4 kept replies (%d)", n);
  NOEXC(Java_akka_dispatch_gpu_AgxJni_stageTellsArrays(env, K, eng, td, ts, tp, 1));
  NOEXC(Java_akka_dispatch_gpu_AgxJni_run(env, K, eng, 1 << 30, st));

  /* the lock-free tell path: one pump submission per burst */
  int subs = 0;
  for (jint i = 1; i <= 1000; ++i) subs += Java_akka_dispatch_gpu_AgxJni_tell(env, K, eng, 3000, AGX_NO_SENDER, i) ? 1 : 0;
  CHECK(subs == 1, "a burst of 1000 tells to an idle engine submitted %d pumps (want 1)", subs);
  NOEXC(Java_akka_dispatch_gpu_AgxJni_run(env, K, eng, 1 << 30, st));
  CHECK(!Java_akka_dispatch_gpu_AgxJni_pumpIdle(env, K, eng), "pumpIdle with nothing pending asked for another run");
  NOEXC(Java_akka_dispatch_gpu_AgxJni_readState(env, K, eng, 3000, 1, w, al));
  CHECK(L(w)[0] == 1000 && L(w)[1] == 500500, "burst delivered: count %lld sum %lld", (long long)L(w)[0],
        (long long)L(w)[1]);
  /* 4 sender threads race the pump (this thread): it runs only when a submission is outstanding */
  tell_arg ta[4];
  pthread_t th[4];
  atomic_store(&t_submitted, 0);
  for (int t = 0; t < 4; ++t) {
    ta[t].eng = eng;
    ta[t].t = t;
    pthread_create(&th[t], NULL, teller, &ta[t]);
  }
  long ran = 0;
  int done = 0;
  for (long spin = 0; spin < 200000000L; ++spin) {
    if (atomic_load(&t_submitted) == ran) {
      if (done) break;
      int all = 1;
      for (int t = 0; t < 4; ++t) all &= atomic_load(&ta_done[t]);
      done = all;  /* one more look after every sender finished: a late submission is still run */
      continue;
    }
    ++ran;
    NOEXC(Java_akka_dispatch_gpu_AgxJni_run(env, K, eng, 1 << 30, NULL));
    if (Java_akka_dispatch_gpu_AgxJni_pumpIdle(env, K, eng)) atomic_fetch_add(&t_submitted, 1);
  }
  for (int t = 0; t < 4; ++t) pthread_join(th[t], NULL);
  for (int t = 0; t < 4; ++t) {
    NOEXC(Java_akka_dispatch_gpu_AgxJni_readState(env, K, eng, 3100 + t, 1, w, al));
    CHECK(L(w)[0] == TELLS && L(w)[1] == (long long)TELLS * (TELLS + 1) / 2,
          "thread %d: %lld of %d tells delivered (sum %lld)", t, (long long)L(w)[0], TELLS, (long long)L(w)[1]);
  }
  CHECK(ran >= 1 && ran <= 4 * TELLS, "pump runs %ld", ran);
  NOEXC(Java_akka_dispatch_gpu_AgxJni_getStats(env, K, eng, st));
  CHECK(L(st)[6] == 0, "in flight after the last pump: %lld", (long long)L(st)[6]);
  CHECK(L(st)[4] + L(st)[3] == L(st)[0] + L(st)[1] + L(st)[6], "staged + emitted = delivered + dead + in flight");
  CHECK(!Java_akka_dispatch_gpu_AgxJni_pumpIdle(env, K, eng), "idle after the race");
  CHECK(ran >= 4 * TELLS / MSGCAP, "pump runs %ld: a burst of 6x msg_capacity needs several", ran);
  printf("lock-free tell path: %d threads x %d tells (msg_capacity %d), %ld pump runs\n", 4, TELLS, MSGCAP, ran);

  /* a pump budget of one superstep (gpu.supersteps-per-pump = 1): throughput 5, 100 tells to one
     COUNTER actor need 20 supersteps -- every pump but the last ends with mail in flight and
     pumpIdle answers "run again" (the status stays scheduled: no tell can submit a second pump) */
  int sub1 = 0;
  for (jint i = 1; i <= 100; ++i) sub1 += Java_akka_dispatch_gpu_AgxJni_tell(env, K, eng, 3200, AGX_NO_SENDER, i) ? 1 : 0;
  CHECK(sub1 == 1, "budget burst submitted %d pumps", sub1);
  int pumps = 0, again = 1;
  while (again && pumps < 1000) {
    ++pumps;
    NOEXC(Java_akka_dispatch_gpu_AgxJni_run(env, K, eng, 1, NULL));
    again = Java_akka_dispatch_gpu_AgxJni_pumpIdle(env, K, eng);
    if (again && pumps == 1)
      CHECK(!Java_akka_dispatch_gpu_AgxJni_tell(env, K, eng, 3201, AGX_NO_SENDER, 1), "a tell while the pump is "
            "rescheduled must not submit a second pump");
  }
  NOEXC(Java_akka_dispatch_gpu_AgxJni_readState(env, K, eng, 3200, 1, w, al));
  CHECK(L(w)[0] == 100 && L(w)[1] == 5050, "budgeted pumps delivered %lld of 100", (long long)L(w)[0]);
  NOEXC(Java_akka_dispatch_gpu_AgxJni_readState(env, K, eng, 3201, 1, w, al));
  CHECK(L(w)[0] == 1, "the tell made during the budgeted pumps was delivered (%lld)", (long long)L(w)[0]);
  CHECK(pumps >= 20 && pumps <= 22, "budgeted pumps: %d runs of one superstep for 100 messages at throughput 5", pumps);
  /* the executor rejected the pump: pumpCancel -> idle, the next tell submits */
  CHECK(Java_akka_dispatch_gpu_AgxJni_tell(env, K, eng, 3202, AGX_NO_SENDER, 1), "idle engine: submit");
  NOEXC(Java_akka_dispatch_gpu_AgxJni_pumpCancel(env, K, eng));
  CHECK(Java_akka_dispatch_gpu_AgxJni_tell(env, K, eng, 3202, AGX_NO_SENDER, 2), "after pumpCancel the next tell submits");
  NOEXC(Java_akka_dispatch_gpu_AgxJni_run(env, K, eng, 1 << 30, st));
  CHECK(!Java_akka_dispatch_gpu_AgxJni_pumpIdle(env, K, eng), "idle after the rejected pump's tells ran");
  NOEXC(Java_akka_dispatch_gpu_AgxJni_readState(env, K, eng, 3202, 1, w, al));
  CHECK(L(w)[0] == 2, "both tells around the rejection delivered (%lld)", (long long)L(w)[0]);
  printf("pump budget: %d pumps of one superstep, pumpCancel OK\n", pumps);

  NOEXC(Java_akka_dispatch_gpu_AgxJni_destroy(env, K, eng));
  free_obj(d);
  free_obj(s);
  free_obj(p);
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("jni_harness OK\n");
  return 0;
}

/*
 * jni_caller.c -- runs the JNI glue (jni/rsketch_jni.c) against a fake JVM.
 *
 * No JDK exists in this image, so the glue is compiled against the test
 * double tests/c/jni_mock/jni.h and driven here the way a JVM would drive it:
 * JNI_OnLoad on the "loading" thread, native methods called with an env,
 * jstrings, direct buffers and Completion objects, and RSketchNative.complete
 * (mocked) receiving what the library's completion thread delivers.  Checks:
 *  - JNI_OnLoad resolves RSketchNative and complete(Object,int,int,long,
 *    boolean[]) once (no FindClass on the completion thread);
 *  - completions arrive once each, in submission order, with the reply;
 *  - the completion thread attaches itself (daemon) and a thread that cannot
 *    attach parks its jobs: they are delivered by the next native call on a
 *    Java thread (never dropped);
 *  - a reply array that cannot be allocated fails the future
 *    (RSK_ERR_OUT_OF_MEMORY) and a complete() that throws is called again with
 *    RSK_ERR_DEVICE: every future completes;
 *  - a "listener" that calls back into the natives from inside complete()
 *    (the worst case: RSketchNative.complete hands off to an event loop, but
 *    nothing in the glue may rely on that) neither deadlocks nor breaks order;
 *  - the RBitSet natives, exceptions and the shim's keyspace through JNI.
 * Needs a GPU (librsketch.so does the work); run by tests/test_jni_shim.py.
 */
#include <jni.h>
#include <pthread.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "../../oracle/rsk_oracle.h"
#include "rsketch_diag.h"
#include "rsketch_shim.h"

static int failures;
#define CHECK(cond)                                                  \
  do {                                                               \
    if (!(cond)) {                                                   \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                    \
    }                                                                \
  } while (0)

/* ------------------------------------------------------------ fake JVM */
enum { O_CLASS, O_STRING, O_DIRECT, O_BOOLARR, O_BYTEARR, O_INTARR, O_LONGARR, O_DOUBLEARR, O_OBJARR, O_COMPLETION };

struct mock_obj {
  int kind;
  char *s;       /* O_STRING, O_CLASS (name) */
  void *addr;    /* O_DIRECT */
  int64_t cap;   /* O_DIRECT: capacity in elements */
  int n;         /* arrays */
  void *data;    /* arrays */
  jobject *items; /* O_OBJARR */
  int id;        /* O_COMPLETION */
};
struct mock_method {
  char name[64], sig[64];
};

static struct mock_method g_complete_method;
static int find_class_calls, find_class_rsk;
static __thread int t_attached;
static __thread char t_exc[128];  /* pending exception class ("" = none) */
static __thread char t_exc_msg[256];
static volatile int attach_failures;     /* inject: AttachCurrentThreadAsDaemon fails this many times */
static volatile int bool_array_failures; /* inject: NewBooleanArray returns NULL this many times */
static int globals_live;                 /* global refs outstanding */
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_t main_thread;

static jobject obj(int kind) {
  jobject o = calloc(1, sizeof *o);
  o->kind = kind;
  return o;
}
static jobject jstr(const char *s) {
  jobject o = obj(O_STRING);
  o->s = strdup(s);
  return o;
}
static jobject direct(void *addr, int64_t cap) {
  jobject o = obj(O_DIRECT);
  o->addr = addr;
  o->cap = cap;
  return o;
}

/* completions delivered by "RSketchNative.complete" */
#define MAXC 128
static struct {
  int fired, kind, status, calls;
  int64_t value;
  int on_main, order;
  uint8_t replies[64];
  int nreplies;
} C[MAXC];
static int deliveries;
static int throw_once_id = -1;    /* complete() of this id throws the first time */
static int reenter_id = -1;       /* complete() of this id calls back into the natives */
static pthread_cond_t g_cv = PTHREAD_COND_INITIALIZER;

static void reenter_listener(JNIEnv *env); /* below */

static jclass m_FindClass(JNIEnv *env, const char *name) {
  (void)env;
  find_class_calls++;
  if (strcmp(name, "org/redisson/gpu/RSketchNative") == 0) find_class_rsk++;
  jobject c = obj(O_CLASS);
  c->s = strdup(name);
  return c;
}
static jint m_ThrowNew(JNIEnv *env, jclass c, const char *msg) {
  (void)env;
  snprintf(t_exc, sizeof t_exc, "%s", c->s);
  snprintf(t_exc_msg, sizeof t_exc_msg, "%s", msg ? msg : "");
  return 0;
}
static jboolean m_ExceptionCheck(JNIEnv *env) {
  (void)env;
  return t_exc[0] != 0;
}
static void m_ExceptionClear(JNIEnv *env) {
  (void)env;
  t_exc[0] = 0;
}
static jobject m_NewGlobalRef(JNIEnv *env, jobject o) {
  (void)env;
  pthread_mutex_lock(&g_mu);
  globals_live++;
  pthread_mutex_unlock(&g_mu);
  return o;
}
static void m_DeleteGlobalRef(JNIEnv *env, jobject o) {
  (void)env;
  (void)o;
  pthread_mutex_lock(&g_mu);
  globals_live--;
  pthread_mutex_unlock(&g_mu);
}
static void m_DeleteLocalRef(JNIEnv *env, jobject o) {
  (void)env;
  (void)o;
}
static jmethodID m_GetStaticMethodID(JNIEnv *env, jclass c, const char *name, const char *sig) {
  (void)env;
  (void)c;
  snprintf(g_complete_method.name, sizeof g_complete_method.name, "%s", name);
  snprintf(g_complete_method.sig, sizeof g_complete_method.sig, "%s", sig);
  return &g_complete_method;
}
/* RSketchNative.complete(Object target, int kind, int status, long value, boolean[] replies) */
static void m_CallStaticVoidMethod(JNIEnv *env, jclass c, jmethodID m, ...) {
  (void)c;
  va_list ap;
  va_start(ap, m);
  jobject target = va_arg(ap, jobject);
  jint kind = va_arg(ap, jint);
  jint status = va_arg(ap, jint);
  jlong value = va_arg(ap, jlong);
  jobject arr = va_arg(ap, jobject);
  va_end(ap);
  const int id = target->id;
  pthread_mutex_lock(&g_mu);
  C[id].calls++;
  const int throw_now = id == throw_once_id && C[id].calls == 1;
  if (!throw_now) {
    C[id].fired++;
    C[id].kind = kind;
    C[id].status = status;
    C[id].value = value;
    C[id].on_main = pthread_equal(pthread_self(), main_thread);
    C[id].order = ++deliveries;
    C[id].nreplies = arr ? (arr->n < 64 ? arr->n : 64) : -1;
    if (arr) memcpy(C[id].replies, arr->data, (size_t)(C[id].nreplies));
  }
  pthread_cond_broadcast(&g_cv);
  pthread_mutex_unlock(&g_mu);
  if (throw_now) {
    snprintf(t_exc, sizeof t_exc, "java/lang/RuntimeException");
    return;
  }
  if (id == reenter_id) reenter_listener(env);
}
static const char *m_GetStringUTFChars(JNIEnv *env, jstring s, jboolean *copy) {
  (void)env;
  if (copy) *copy = 0;
  return s->s;
}
static void m_ReleaseStringUTFChars(JNIEnv *env, jstring s, const char *c) {
  (void)env;
  (void)s;
  (void)c;
}
static jsize m_GetArrayLength(JNIEnv *env, jarray a) {
  (void)env;
  return a->n;
}
static jobject m_GetObjectArrayElement(JNIEnv *env, jobjectArray a, jsize i) {
  (void)env;
  return a->items[i];
}
static jobject new_array(int kind, jsize n, size_t elem) {
  jobject a = obj(kind);
  a->n = n;
  a->data = calloc((size_t)(n > 0 ? n : 1), elem);
  return a;
}
static jbooleanArray m_NewBooleanArray(JNIEnv *env, jsize n) {
  (void)env;
  pthread_mutex_lock(&g_mu);
  const int fail = bool_array_failures > 0;
  if (fail) bool_array_failures--;
  pthread_mutex_unlock(&g_mu);
  if (fail) {
    snprintf(t_exc, sizeof t_exc, "java/lang/OutOfMemoryError");
    return NULL;
  }
  return new_array(O_BOOLARR, n, 1);
}
static void m_SetBooleanArrayRegion(JNIEnv *env, jbooleanArray a, jsize at, jsize n, const jboolean *v) {
  (void)env;
  memcpy((jboolean *)a->data + at, v, (size_t)n);
}
static jbyteArray m_NewByteArray(JNIEnv *env, jsize n) {
  (void)env;
  return new_array(O_BYTEARR, n, 1);
}
static void m_SetByteArrayRegion(JNIEnv *env, jbyteArray a, jsize at, jsize n, const jbyte *v) {
  (void)env;
  memcpy((jbyte *)a->data + at, v, (size_t)n);
}
static void m_GetByteArrayRegion(JNIEnv *env, jbyteArray a, jsize at, jsize n, jbyte *v) {
  (void)env;
  memcpy(v, (jbyte *)a->data + at, (size_t)n);
}
static void m_GetIntArrayRegion(JNIEnv *env, jintArray a, jsize at, jsize n, jint *v) {
  (void)env;
  memcpy(v, (jint *)a->data + at, sizeof(jint) * (size_t)n);
}
static void m_GetLongArrayRegion(JNIEnv *env, jlongArray a, jsize at, jsize n, jlong *v) {
  (void)env;
  memcpy(v, (jlong *)a->data + at, sizeof(jlong) * (size_t)n);
}
static void m_SetLongArrayRegion(JNIEnv *env, jlongArray a, jsize at, jsize n, const jlong *v) {
  (void)env;
  memcpy((jlong *)a->data + at, v, sizeof(jlong) * (size_t)n);
}
static void m_SetDoubleArrayRegion(JNIEnv *env, jdoubleArray a, jsize at, jsize n, const jdouble *v) {
  (void)env;
  memcpy((jdouble *)a->data + at, v, sizeof(jdouble) * (size_t)n);
}
static void *m_GetDirectBufferAddress(JNIEnv *env, jobject b) {
  (void)env;
  return b && b->kind == O_DIRECT ? b->addr : NULL;
}
static jlong m_GetDirectBufferCapacity(JNIEnv *env, jobject b) {
  (void)env;
  return b && b->kind == O_DIRECT ? b->cap : -1;
}

static const struct JNINativeInterface_ g_fns = {
    m_FindClass,          m_ThrowNew,           m_ExceptionCheck,        m_ExceptionClear,
    m_NewGlobalRef,       m_DeleteGlobalRef,    m_DeleteLocalRef,        m_GetStaticMethodID,
    m_CallStaticVoidMethod, m_GetStringUTFChars, m_ReleaseStringUTFChars, m_GetArrayLength,
    m_GetObjectArrayElement, m_NewBooleanArray, m_SetBooleanArrayRegion, m_NewByteArray,
    m_SetByteArrayRegion, m_GetByteArrayRegion, m_GetIntArrayRegion,     m_GetLongArrayRegion,
    m_SetLongArrayRegion, m_SetDoubleArrayRegion, m_GetDirectBufferAddress, m_GetDirectBufferCapacity,
};
static JNIEnv g_env = &g_fns;

static jint vm_GetEnv(JavaVM *vm, void **env, jint version) {
  (void)vm;
  (void)version;
  if (!t_attached) return JNI_EDETACHED;
  *env = &g_env;
  return JNI_OK;
}
static jint vm_Attach(JavaVM *vm, void **env, void *args) {
  (void)vm;
  (void)args;
  pthread_mutex_lock(&g_mu);
  const int fail = attach_failures > 0;
  if (fail) attach_failures--;
  pthread_mutex_unlock(&g_mu);
  if (fail) return JNI_ERR;
  t_attached = 1;
  *env = &g_env;
  return JNI_OK;
}
static const struct JNIInvokeInterface_ g_vmfns = {vm_GetEnv, vm_Attach};
static JavaVM g_vm = &g_vmfns;

/* --------------------------------------------- the glue's exported natives */
#define N(ret, name) JNIEXPORT ret JNICALL Java_org_redisson_gpu_RSketchNative_##name
jint JNI_OnLoad(JavaVM *vm, void *reserved);
N(jlong, init)(JNIEnv *, jclass, jint, jboolean);
N(void, shutdown)(JNIEnv *, jclass, jlong);
N(void, sync)(JNIEnv *, jclass, jlong);
N(void, reap)(JNIEnv *, jclass);
N(jint, type)(JNIEnv *, jclass, jlong, jstring);
N(jboolean, hllAdd)(JNIEnv *, jclass, jlong, jstring, jobject, jobject, jlong);
N(jlong, hllCount)(JNIEnv *, jclass, jlong, jstring);
N(void, hllAddAsync)(JNIEnv *, jclass, jlong, jstring, jobject, jobject, jlong, jobject);
N(void, hllCountAsync)(JNIEnv *, jclass, jlong, jstring, jobject);
N(jboolean, bloomTryInit)(JNIEnv *, jclass, jlong, jstring, jlong, jdouble, jlongArray, jdoubleArray);
N(void, bloomAddAsync)(JNIEnv *, jclass, jlong, jstring, jlong, jint, jobject, jobject, jlong, jobject);
N(jbooleanArray, bloomContains)(JNIEnv *, jclass, jlong, jstring, jlong, jint, jobject, jobject, jlong);
N(jbyteArray, bitsetGet)(JNIEnv *, jclass, jlong, jstring);
N(void, bitsetSetBits)(JNIEnv *, jclass, jlong, jstring, jlongArray, jboolean);
N(jlong, bitsetCardinality)(JNIEnv *, jclass, jlong, jstring);

static jlong SPACE;
static jclass CLS;

/* A batch of n 16-byte keys as the Java side passes it (KeyBuffer: direct
 * ByteBuffer + LongBuffer of n+1 offsets). */
typedef struct {
  jobject keys, offs;
  unsigned char *k;
  int64_t *o;
} jbatch;
static jbatch keys16(uint64_t seed, int64_t n) {
  jbatch b;
  b.k = malloc((size_t)n * 16);
  b.o = malloc((size_t)(n + 1) * 8);
  orc_gen_keys16(seed, 0, (uint64_t)n, b.k);
  for (int64_t i = 0; i <= n; ++i) b.o[i] = 16 * i;
  b.keys = direct(b.k, 16 * n);
  b.offs = direct(b.o, n + 1);
  return b;
}
static jobject completion(int id) {
  jobject o = obj(O_COMPLETION);
  o->id = id;
  return o;
}
static void wait_fired(int id) {
  pthread_mutex_lock(&g_mu);
  struct timespec until;
  clock_gettime(CLOCK_REALTIME, &until);
  until.tv_sec += 60;
  while (C[id].fired == 0)
    if (pthread_cond_timedwait(&g_cv, &g_mu, &until)) break;
  pthread_mutex_unlock(&g_mu);
}

static jbatch REB;
/* a "listener" that runs inline on the completion thread and calls back in */
static void reenter_listener(JNIEnv *env) {
  jobject nm = jstr("jhll");
  const jlong c = Java_org_redisson_gpu_RSketchNative_hllCount(env, CLS, SPACE, nm);
  CHECK(!m_ExceptionCheck(env) && c > 0);
  Java_org_redisson_gpu_RSketchNative_hllAddAsync(env, CLS, SPACE, nm, REB.keys, REB.offs, 1000, completion(61));
  CHECK(!m_ExceptionCheck(env));
}

static void on_alarm(int sig) {
  (void)sig;
  static const char msg[] = "FAIL watchdog: deadlock\n";
  (void)!write(2, msg, sizeof msg - 1);
  _exit(3);
}

int main(void) {
  signal(SIGALRM, on_alarm);
  alarm(100);
  main_thread = pthread_self();
  t_attached = 1; /* the JVM's own thread */
  JNIEnv *env = &g_env;
  CLS = m_FindClass(env, "org/redisson/gpu/RSketchNative");
  find_class_calls = find_class_rsk = 0;

  /* System.loadLibrary inside RSketchNative's static initializer */
  CHECK(JNI_OnLoad(&g_vm, NULL) == JNI_VERSION_1_6);
  CHECK(find_class_rsk == 1 && strcmp(g_complete_method.name, "complete") == 0 &&
        strcmp(g_complete_method.sig, "(Ljava/lang/Object;IIJ[Z)V") == 0);
  const int finds_after_load = find_class_calls;

  SPACE = Java_org_redisson_gpu_RSketchNative_init(env, CLS, 0, JNI_FALSE);
  CHECK(SPACE != 0 && !m_ExceptionCheck(env));

  /* async adds: delivered once each, in submission order, off the Java thread */
  jbatch b = keys16(0x5EED0300, 100000);
  REB = keys16(0x5EED0301, 1000);
  jobject nm = jstr("jhll");
  for (int i = 0; i < 20; ++i) /* first creates the key, the rest change nothing */
    Java_org_redisson_gpu_RSketchNative_hllAddAsync(env, CLS, SPACE, nm, b.keys, b.offs, 100000, completion(i));
  CHECK(!m_ExceptionCheck(env));
  Java_org_redisson_gpu_RSketchNative_sync(env, CLS, SPACE);
  for (int i = 0; i < 20; ++i) {
    CHECK(C[i].fired == 1 && C[i].status == 0 && C[i].kind == 0 && C[i].value == (i == 0));
    CHECK(!C[i].on_main);
    if (i) CHECK(C[i].order == C[i - 1].order + 1);
  }
  uint8_t *regs = calloc(16384, 1);
  orc_hll_add_raw(regs, b.k, NULL, 16, 100000);
  const uint64_t want = orc_hll_count_dense_regs(regs);
  Java_org_redisson_gpu_RSketchNative_hllCountAsync(env, CLS, SPACE, nm, completion(20));
  wait_fired(20);
  CHECK(C[20].fired == 1 && C[20].kind == 1 && (uint64_t)C[20].value == want);
  CHECK(find_class_calls == finds_after_load); /* the completion thread looked nothing up */

  /* a completion thread that cannot attach (a second context: its completion
   * thread has never been attached): parked, delivered by the next native call */
  {
    const jlong space2 = Java_org_redisson_gpu_RSketchNative_init(env, CLS, 0, JNI_FALSE);
    CHECK(space2 != 0);
    attach_failures = 1000;
    Java_org_redisson_gpu_RSketchNative_hllAddAsync(env, CLS, space2, nm, b.keys, b.offs, 100000, completion(21));
    Java_org_redisson_gpu_RSketchNative_hllCountAsync(env, CLS, space2, nm, completion(22));
    /* rsk_shim_sync returns after the callbacks ran (they parked the jobs); sync then reaps */
    Java_org_redisson_gpu_RSketchNative_sync(env, CLS, space2);
    CHECK(C[21].fired == 1 && C[21].status == 0 && C[21].value == 1 && C[21].on_main);
    CHECK(C[22].fired == 1 && C[22].status == 0 && (uint64_t)C[22].value == want && C[22].on_main);
    CHECK(C[22].order == C[21].order + 1); /* parked jobs keep submission order */
    attach_failures = 0;
    Java_org_redisson_gpu_RSketchNative_shutdown(env, CLS, space2);
  }

  /* a reply array that cannot be allocated, and a complete() that throws */
  {
    jobject bn = jstr("jbloom");
    jlongArray cfg = new_array(O_LONGARR, 3, 8);
    CHECK(Java_org_redisson_gpu_RSketchNative_bloomTryInit(env, CLS, SPACE, bn, 1000, 0.01, cfg, NULL) == JNI_TRUE);
    const jlong size = ((jlong *)cfg->data)[0];
    const jint k = (jint)((jlong *)cfg->data)[1];
    jbatch bb = keys16(0x5EED0302, 40);
    bool_array_failures = 1;
    Java_org_redisson_gpu_RSketchNative_bloomAddAsync(env, CLS, SPACE, bn, size, k, bb.keys, bb.offs, 40, completion(30));
    wait_fired(30);
    CHECK(C[30].fired == 1 && C[30].status == 6 && C[30].nreplies == -1); /* RSK_ERR_OUT_OF_MEMORY */
    throw_once_id = 31;
    Java_org_redisson_gpu_RSketchNative_bloomAddAsync(env, CLS, SPACE, bn, size, k, bb.keys, bb.offs, 40, completion(31));
    wait_fired(31);
    CHECK(C[31].calls == 2 && C[31].fired == 1 && C[31].status == 5); /* re-sent as RSK_ERR_DEVICE */
    Java_org_redisson_gpu_RSketchNative_bloomAddAsync(env, CLS, SPACE, bn, size, k, bb.keys, bb.offs, 40, completion(32));
    wait_fired(32);
    CHECK(C[32].fired == 1 && C[32].status == 0 && C[32].kind == 3 && C[32].nreplies == 40);
    int none = 1; /* every key was added before: every reply false */
    for (int i = 0; i < 40; ++i) none &= C[32].replies[i] == 0;
    CHECK(none);
    jbooleanArray got = Java_org_redisson_gpu_RSketchNative_bloomContains(env, CLS, SPACE, bn, size, k, bb.keys, bb.offs, 40);
    CHECK(got && got->n == 40);
    int all = 1;
    for (int i = 0; got && i < 40; ++i) all &= ((uint8_t *)got->data)[i] == 1;
    CHECK(all);
    /* getBitSet(bloomName) through JNI: GET = the filter's bits */
    jbyteArray bytes = Java_org_redisson_gpu_RSketchNative_bitsetGet(env, CLS, SPACE, bn);
    CHECK(bytes && bytes->n > 0 && bytes->n <= (size + 7) / 8);
    uint8_t *obits = calloc((size_t)((size + 7) / 8), 1);
    orc_bloom_add_batch(obits, size, k, bb.k, NULL, 16, 40, NULL);
    CHECK(bytes && memcmp(bytes->data, obits, (size_t)bytes->n) == 0);
    int64_t pc = 0;
    for (int64_t i = 0; i < (size + 7) / 8; ++i) pc += __builtin_popcount(obits[i]);
    CHECK(Java_org_redisson_gpu_RSketchNative_bitsetCardinality(env, CLS, SPACE, bn) == pc);
    free(obits);
  }

  /* a listener calling back into the natives from the completion thread */
  reenter_id = 60;
  Java_org_redisson_gpu_RSketchNative_hllAddAsync(env, CLS, SPACE, nm, REB.keys, REB.offs, 1000, completion(60));
  wait_fired(60);
  wait_fired(61);
  Java_org_redisson_gpu_RSketchNative_sync(env, CLS, SPACE);
  CHECK(C[60].fired == 1 && C[60].status == 0 && C[60].value == 1);
  CHECK(C[61].fired == 1 && C[61].status == 0 && C[61].value == 0 && C[61].order > C[60].order);

  /* RBitSet natives: missing name -> null; SETBIT / GET; wrong type -> RedisException */
  {
    jobject bs = jstr("jbits");
    CHECK(Java_org_redisson_gpu_RSketchNative_bitsetGet(env, CLS, SPACE, bs) == NULL && !m_ExceptionCheck(env));
    jlongArray idx = new_array(O_LONGARR, 2, 8);
    ((jlong *)idx->data)[0] = 0;
    ((jlong *)idx->data)[1] = 9;
    Java_org_redisson_gpu_RSketchNative_bitsetSetBits(env, CLS, SPACE, bs, idx, JNI_TRUE);
    jbyteArray v = Java_org_redisson_gpu_RSketchNative_bitsetGet(env, CLS, SPACE, bs);
    CHECK(v && v->n == 2 && ((uint8_t *)v->data)[0] == 0x80 && ((uint8_t *)v->data)[1] == 0x40);
    ((jlong *)idx->data)[0] = -5;
    Java_org_redisson_gpu_RSketchNative_bitsetSetBits(env, CLS, SPACE, bs, idx, JNI_TRUE);
    CHECK(m_ExceptionCheck(env) && strcmp(t_exc, "org/redisson/client/RedisException") == 0 &&
          strstr(t_exc_msg, "bit offset") != NULL);
    m_ExceptionClear(env);
    CHECK(Java_org_redisson_gpu_RSketchNative_bitsetCardinality(env, CLS, SPACE, nm) == 0 && m_ExceptionCheck(env) &&
          strcmp(t_exc, "org/redisson/client/RedisException") == 0); /* an HLL name: WRONGTYPE */
    m_ExceptionClear(env);
    CHECK(Java_org_redisson_gpu_RSketchNative_hllCount(env, CLS, SPACE, jstr("jbloom")) == 0 && m_ExceptionCheck(env));
    m_ExceptionClear(env);
    CHECK(Java_org_redisson_gpu_RSketchNative_type(env, CLS, SPACE, bs) == 3);
  }

  /* a context marked dead (as after a device error on its streams): every call
   * and sync() throw RedisException, and the native shutdown that
   * GpuSketchContext.shutdown() runs in its finally still releases it */
  {
    const jlong space3 = Java_org_redisson_gpu_RSketchNative_init(env, CLS, 0, JNI_FALSE);
    CHECK(space3 != 0);
    Java_org_redisson_gpu_RSketchNative_hllAddAsync(env, CLS, space3, nm, REB.keys, REB.offs, 1000, completion(70));
    Java_org_redisson_gpu_RSketchNative_sync(env, CLS, space3);
    CHECK(C[70].fired == 1 && C[70].status == 0);
    CHECK(rsk_diag_mark_dead(rsk_shim_context((int64_t)space3)) == RSK_OK);
    CHECK(Java_org_redisson_gpu_RSketchNative_hllCount(env, CLS, space3, nm) == 0 && m_ExceptionCheck(env) &&
          strcmp(t_exc, "org/redisson/client/RedisException") == 0);
    m_ExceptionClear(env);
    Java_org_redisson_gpu_RSketchNative_sync(env, CLS, space3); /* try { sync } ... */
    CHECK(m_ExceptionCheck(env) && strcmp(t_exc, "org/redisson/client/RedisException") == 0);
    m_ExceptionClear(env);
    Java_org_redisson_gpu_RSketchNative_shutdown(env, CLS, space3); /* ... finally { shutdown } */
    CHECK(!m_ExceptionCheck(env));
  }

  Java_org_redisson_gpu_RSketchNative_shutdown(env, CLS, SPACE);
  CHECK(!m_ExceptionCheck(env));
  CHECK(globals_live == 1); /* only the class reference JNI_OnLoad keeps */
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("jni_caller ok\n");
  return 0;
}

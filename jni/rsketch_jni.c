/*
 * rsketch_jni.c -- JNI glue of org.redisson.gpu.RSketchNative
 * (jni/java/org/redisson/gpu/RSketchNative.java) over rsketch_shim.c.
 *
 * Needs a JDK's jni.h, which this image lacks: it is source here and is built
 * where JAVA_HOME exists (make -C jni jni).  Every method follows one pattern:
 * fetch names / direct-buffer addresses and capacities, call the shim, throw
 * rsk_shim_exception_class(rc) with rsk_shim_last_error() on failure.  The
 * shim (all checks, the name -> object keyspace, the config guard) is what
 * tests/c/shim_caller.c runs on the GPU.
 *
 * Async methods take a Completion (RSketchNative.java: the Netty promise and
 * the executor its listeners run on).  The shim's callback runs on the
 * library's completion thread: it attaches that thread to the JVM once (as a
 * daemon), and calls RSketchNative.complete(completion, kind, status, value,
 * replies), which only hands the result to the completion's executor -- the
 * Netty event loop GpuSketchContext pinned, as a Redis reply is decoded and
 * its promise completed on a connection's event loop
 * (CommandAsyncService.java:86-105) -- so user listeners never run on the
 * library's thread.  The class and method are resolved once, in JNI_OnLoad
 * (which runs inside RSketchNative's static initializer, so FindClass sees the
 * class loader that loaded the binding: a natively attached thread would only
 * see the system loader).  A result is never dropped: if the completion
 * thread cannot attach, the job is parked and delivered by the next native
 * call (or RSketchNative.reap) on any Java thread.
 */
#include <jni.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "rsketch_shim.h"

static JavaVM *g_vm;
static jclass g_native;      /* global ref: org.redisson.gpu.RSketchNative */
static jmethodID g_complete; /* static void complete(Object, int, int, long, boolean[]) */

static void reap(JNIEnv *env); /* delivers parked completions (below) */

JNIEXPORT jint JNICALL JNI_OnLoad(JavaVM *vm, void *reserved) {
  (void)reserved;
  JNIEnv *env = NULL;
  if ((*vm)->GetEnv(vm, (void **)&env, JNI_VERSION_1_6) != JNI_OK) return JNI_ERR;
  jclass c = (*env)->FindClass(env, "org/redisson/gpu/RSketchNative");
  if (!c) return JNI_ERR; /* NoClassDefFoundError pending: System.loadLibrary fails */
  g_native = (jclass)(*env)->NewGlobalRef(env, c);
  (*env)->DeleteLocalRef(env, c);
  if (!g_native) return JNI_ERR;
  g_complete = (*env)->GetStaticMethodID(env, g_native, "complete", "(Ljava/lang/Object;IIJ[Z)V");
  if (!g_complete) return JNI_ERR;
  g_vm = vm;
  return JNI_VERSION_1_6;
}

JNIEXPORT void JNICALL JNI_OnUnload(JavaVM *vm, void *reserved) {
  (void)reserved;
  JNIEnv *env = NULL;
  if ((*vm)->GetEnv(vm, (void **)&env, JNI_VERSION_1_6) == JNI_OK && g_native) (*env)->DeleteGlobalRef(env, g_native);
  g_native = NULL;
  g_complete = NULL;
}

static rsk_shim_buf direct(JNIEnv *env, jobject buf) {
  rsk_shim_buf b = {NULL, 0};
  if (buf) {
    b.addr = (*env)->GetDirectBufferAddress(env, buf);
    b.cap = b.addr ? (int64_t)(*env)->GetDirectBufferCapacity(env, buf) : 0;
  }
  return b;
}

/* Returns 1 (and leaves a pending exception) when rc is an error. */
static int raise(JNIEnv *env, int rc) {
  const char *cls = rsk_shim_exception_class(rc);
  if (!cls) return 0;
  jclass c = (*env)->FindClass(env, cls);
  if (c) (*env)->ThrowNew(env, c, rsk_shim_last_error());
  return 1;
}

static int throw_iae(JNIEnv *env, const char *msg) {
  jclass c = (*env)->FindClass(env, "java/lang/IllegalArgumentException");
  if (c) (*env)->ThrowNew(env, c, msg);
  return 1;
}

/* A Java String as modified UTF-8 (NULL with a pending exception on failure). */
typedef struct {
  jstring s;
  const char *c;
} jname;

static int name_get(JNIEnv *env, jstring s, jname *out) {
  out->s = s;
  out->c = NULL;
  if (!s) return throw_iae(env, "name is null");
  out->c = (*env)->GetStringUTFChars(env, s, NULL);
  return out->c == NULL; /* OutOfMemoryError pending */
}
static void name_put(JNIEnv *env, jname *n) {
  if (n->c) (*env)->ReleaseStringUTFChars(env, n->s, n->c);
}

/* String[] -> const char *[] (at most 4096 names). */
typedef struct {
  int k;
  jname *ns;
  const char **cs;
} jnames;

/* 0 on success; 1 with a pending exception. */
static int names_get(JNIEnv *env, jobjectArray arr, jnames *out) {
  out->k = 0;
  out->ns = NULL;
  out->cs = NULL;
  if (!arr) return throw_iae(env, "names is null");
  const jsize k = (*env)->GetArrayLength(env, arr);
  if (k > 4096) return throw_iae(env, "at most 4096 keys per call");
  out->ns = calloc((size_t)(k > 0 ? k : 1), sizeof(jname));
  out->cs = calloc((size_t)(k > 0 ? k : 1), sizeof(const char *));
  if (!out->ns || !out->cs) {
    free(out->ns);
    free(out->cs);
    out->ns = NULL;
    out->cs = NULL;
    jclass c = (*env)->FindClass(env, "java/lang/OutOfMemoryError");
    if (c) (*env)->ThrowNew(env, c, "names");
    return 1;
  }
  for (jsize i = 0; i < k; ++i) {
    if (name_get(env, (jstring)(*env)->GetObjectArrayElement(env, arr, i), &out->ns[i])) {
      out->k = (int)i;
      return 1;
    }
    out->cs[i] = out->ns[i].c;
  }
  out->k = (int)k;
  return 0;
}
static void names_put(JNIEnv *env, jnames *n) {
  for (int i = 0; i < n->k; ++i) name_put(env, &n->ns[i]);
  free(n->ns);
  free(n->cs);
  n->ns = NULL;
  n->cs = NULL;
  n->k = 0;
}

#define JNI_FN(ret, name) JNIEXPORT ret JNICALL Java_org_redisson_gpu_RSketchNative_##name

JNI_FN(jlong, init)(JNIEnv *env, jclass cls, jint device, jboolean extended) {
  (void)cls;
  reap(env);
  int64_t s = 0;
  return raise(env, rsk_shim_init(device, extended ? 1 : 0, &s)) ? 0 : (jlong)s;
}

JNI_FN(void, shutdown)(JNIEnv *env, jclass cls, jlong space) {
  (void)cls;
  reap(env);
  raise(env, rsk_shim_shutdown(space));
}

JNI_FN(jint, type)(JNIEnv *env, jclass cls, jlong space, jstring name) {
  (void)cls;
  reap(env);
  jname n;
  if (name_get(env, name, &n)) return 0;
  int32_t t = 0;
  int64_t h = 0;
  const int rc = rsk_shim_lookup(space, n.c, &t, &h);
  name_put(env, &n);
  return raise(env, rc) ? 0 : (jint)t;
}

JNI_FN(jboolean, delete)(JNIEnv *env, jclass cls, jlong space, jstring name) {
  (void)cls;
  reap(env);
  jname n;
  if (name_get(env, name, &n)) return JNI_FALSE;
  int32_t d = 0;
  const int rc = rsk_shim_delete(space, n.c, &d);
  name_put(env, &n);
  return raise(env, rc) ? JNI_FALSE : (d ? JNI_TRUE : JNI_FALSE);
}

JNI_FN(jboolean, rename)(JNIEnv *env, jclass cls, jlong space, jstring oldName, jstring newName, jboolean nx) {
  (void)cls;
  reap(env);
  jname a, b;
  if (name_get(env, oldName, &a)) return JNI_FALSE;
  if (name_get(env, newName, &b)) {
    name_put(env, &a);
    return JNI_FALSE;
  }
  int32_t done = 0;
  const int rc = rsk_shim_rename(space, a.c, b.c, nx ? 1 : 0, &done);
  name_put(env, &b);
  name_put(env, &a);
  return raise(env, rc) ? JNI_FALSE : (done ? JNI_TRUE : JNI_FALSE);
}

/* ------------------------------------------------------------------ HLL */
JNI_FN(jboolean, hllAdd)(JNIEnv *env, jclass cls, jlong space, jstring name, jobject keys, jobject offsets, jlong n) {
  (void)cls;
  reap(env);
  jname nm;
  if (name_get(env, name, &nm)) return JNI_FALSE;
  uint8_t changed = 0;
  const int rc = rsk_shim_hll_add(space, nm.c, direct(env, keys), direct(env, offsets), n, &changed);
  name_put(env, &nm);
  if (raise(env, rc)) return JNI_FALSE;
  return changed ? JNI_TRUE : JNI_FALSE;
}

/* Replies into a fresh boolean[] (jboolean is an unsigned byte): the shim
 * writes a C buffer, copied with SetBooleanArrayRegion (no pinned array
 * element pointers to check or release). */
static jbooleanArray replies_array(JNIEnv *env, const uint8_t *r, jlong n) {
  jbooleanArray arr = (*env)->NewBooleanArray(env, (jsize)n);
  if (arr && n) (*env)->SetBooleanArrayRegion(env, arr, 0, (jsize)n, (const jboolean *)r);
  return arr;
}

static uint8_t *reply_buf(JNIEnv *env, jlong n) {
  if (n < 0 || n > 0x7fffffff) {
    throw_iae(env, "batch larger than 2^31 - 1 elements");
    return NULL;
  }
  uint8_t *r = malloc((size_t)(n > 0 ? n : 1));
  if (!r) {
    jclass c = (*env)->FindClass(env, "java/lang/OutOfMemoryError");
    if (c) (*env)->ThrowNew(env, c, "reply buffer");
  }
  return r;
}

JNI_FN(jbooleanArray, hllAddEach)(JNIEnv *env, jclass cls, jlong space, jstring name, jobject keys, jobject offsets,
                                  jlong n) {
  (void)cls;
  reap(env);
  uint8_t *r = reply_buf(env, n);
  if (!r) return NULL;
  jname nm;
  if (name_get(env, name, &nm)) {
    free(r);
    return NULL;
  }
  const int rc = rsk_shim_hll_add_each(space, nm.c, direct(env, keys), direct(env, offsets), n, r, n);
  name_put(env, &nm);
  jbooleanArray arr = raise(env, rc) ? NULL : replies_array(env, r, n);
  free(r);
  return arr;
}

JNI_FN(jlong, hllCount)(JNIEnv *env, jclass cls, jlong space, jstring name) {
  (void)cls;
  reap(env);
  jname nm;
  if (name_get(env, name, &nm)) return 0;
  int64_t v = 0;
  const int rc = rsk_shim_hll_count(space, nm.c, &v);
  name_put(env, &nm);
  return raise(env, rc) ? 0 : (jlong)v;
}

JNI_FN(jlong, hllCountWith)(JNIEnv *env, jclass cls, jlong space, jobjectArray names) {
  (void)cls;
  reap(env);
  jnames ns;
  if (names_get(env, names, &ns)) {
    names_put(env, &ns);
    return 0;
  }
  int64_t v = 0;
  const int rc = rsk_shim_hll_count_with(space, ns.cs, ns.k, &v);
  names_put(env, &ns);
  return raise(env, rc) ? 0 : (jlong)v;
}

JNI_FN(void, hllMergeWith)(JNIEnv *env, jclass cls, jlong space, jstring dst, jobjectArray srcs) {
  (void)cls;
  reap(env);
  jname d;
  if (name_get(env, dst, &d)) return;
  jnames ns;
  if (names_get(env, srcs, &ns)) {
    names_put(env, &ns);
    name_put(env, &d);
    return;
  }
  const int rc = rsk_shim_hll_merge_with(space, d.c, ns.cs, ns.k);
  names_put(env, &ns);
  name_put(env, &d);
  raise(env, rc);
}

JNI_FN(jbooleanArray, batchHllAdd)(JNIEnv *env, jclass cls, jlong space, jobjectArray names, jintArray nameOf,
                                   jobject keys, jobject offsets, jlong n) {
  (void)cls;
  reap(env);
  if (!nameOf || (*env)->GetArrayLength(env, nameOf) < n) {
    throw_iae(env, "nameOf shorter than the batch");
    return NULL;
  }
  uint8_t *r = reply_buf(env, n);
  if (!r) return NULL;
  int32_t *of = malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
  if (!of) {
    free(r);
    return NULL;
  }
  if (n) (*env)->GetIntArrayRegion(env, nameOf, 0, (jsize)n, (jint *)of);
  jnames ns;
  jbooleanArray arr = NULL;
  if (!names_get(env, names, &ns)) {
    const int rc = rsk_shim_batch_hll_add(space, ns.cs, ns.k, of, direct(env, keys), direct(env, offsets), n, r, n);
    if (!raise(env, rc)) arr = replies_array(env, r, n);
  }
  names_put(env, &ns);
  free(of);
  free(r);
  return arr;
}

/* --------------------------------------------------------------- async */
enum { K_BOOL = 0, K_LONG = 1, K_VOID = 2, K_ARRAY = 3 };

typedef struct job {
  jobject target; /* global reference: the RSketchNative.Completion */
  int kind;
  uint8_t *out; /* K_ARRAY: the replies, n bytes */
  int64_t n;
  int status; /* the result, kept while the job waits to be delivered */
  uint64_t value;
  struct job *next;
} job;

/* Jobs whose completion thread could not attach to the JVM: delivered by the
 * next native call on a Java thread (reap), never dropped. */
static pthread_mutex_t g_park_mu = PTHREAD_MUTEX_INITIALIZER;
static job *g_parked;
static volatile int g_parked_n;

/* Completes one job through Java and frees it.  The replies array is made
 * here; if that fails (OutOfMemoryError) the job completes with
 * RSK_ERR_OUT_OF_MEMORY instead, and if complete() itself throws, once more
 * with RSK_ERR_DEVICE -- the future always completes. */
static void deliver(JNIEnv *env, job *j) {
  int status = j->status;
  jbooleanArray arr = NULL;
  if (j->kind == K_ARRAY && status == RSK_OK) {
    arr = replies_array(env, j->out, j->n);
    if (!arr) {
      (*env)->ExceptionClear(env);
      status = RSK_ERR_OUT_OF_MEMORY;
    }
  }
  (*env)->CallStaticVoidMethod(env, g_native, g_complete, j->target, (jint)j->kind, (jint)status,
                               (jlong)j->value, arr);
  if ((*env)->ExceptionCheck(env)) {
    (*env)->ExceptionClear(env);
    (*env)->CallStaticVoidMethod(env, g_native, g_complete, j->target, (jint)j->kind, (jint)RSK_ERR_DEVICE,
                                 (jlong)0, (jbooleanArray)NULL);
    if ((*env)->ExceptionCheck(env)) (*env)->ExceptionClear(env);
  }
  if (arr) (*env)->DeleteLocalRef(env, arr);
  (*env)->DeleteGlobalRef(env, j->target);
  free(j->out);
  free(j);
}

/* Delivers parked jobs (a Java thread, at the top of every native method). */
static void reap(JNIEnv *env) {
  if (!g_parked_n) return;
  pthread_mutex_lock(&g_park_mu);
  job *j = g_parked;
  g_parked = NULL;
  g_parked_n = 0;
  pthread_mutex_unlock(&g_park_mu);
  while (j) { /* parked newest first: deliver in submission order */
    job *rev = NULL;
    while (j) {
      job *nx = j->next;
      j->next = rev;
      rev = j;
      j = nx;
    }
    j = rev;
    while (j) {
      job *nx = j->next;
      deliver(env, j);
      j = nx;
    }
  }
}

/* The shim's callback, on the library's completion thread (or the calling
 * thread for an answer known at once).  The thread is attached once, as a
 * daemon, and stays attached (the completion thread lives as long as the
 * context). */
static void jni_done(void *user, int status, uint64_t value) {
  job *j = user;
  j->status = status;
  j->value = value;
  JNIEnv *env = NULL;
  if ((*g_vm)->GetEnv(g_vm, (void **)&env, JNI_VERSION_1_6) != JNI_OK) {
    env = NULL;
    for (int attempt = 0; attempt < 3 && !env; ++attempt) {
      if ((*g_vm)->AttachCurrentThreadAsDaemon(g_vm, (void **)&env, NULL) != JNI_OK) {
        env = NULL;
        const struct timespec ts = {0, 1000000L << (2 * attempt)}; /* 1, 4, 16 ms */
        nanosleep(&ts, NULL);
      }
    }
  }
  if (!env) { /* park it for the next native call */
    pthread_mutex_lock(&g_park_mu);
    j->next = g_parked;
    g_parked = j;
    g_parked_n = 1;
    pthread_mutex_unlock(&g_park_mu);
    return;
  }
  reap(env); /* earlier parked jobs first: keep submission order */
  deliver(env, j);
}

static job *job_new(JNIEnv *env, jobject target, int kind, int64_t n) {
  if (!target) {
    throw_iae(env, "completion is null");
    return NULL;
  }
  job *j = calloc(1, sizeof *j);
  if (!j) return NULL;
  j->kind = kind;
  j->n = n;
  if (kind == K_ARRAY) {
    j->out = malloc((size_t)(n > 0 ? n : 1));
    if (!j->out) {
      free(j);
      return NULL;
    }
  }
  j->target = (*env)->NewGlobalRef(env, target);
  if (!j->target) {
    free(j->out);
    free(j);
    return NULL;
  }
  return j;
}

/* A call the shim refused never fires: free the job, throw. */
static void job_refused(JNIEnv *env, job *j, int rc) {
  (*env)->DeleteGlobalRef(env, j->target);
  free(j->out);
  free(j);
  raise(env, rc);
}

JNI_FN(void, reap)(JNIEnv *env, jclass cls) {
  (void)cls;
  reap(env);
}

JNI_FN(void, sync)(JNIEnv *env, jclass cls, jlong space) {
  (void)cls;
  reap(env);
  raise(env, rsk_shim_sync(space));
  reap(env);
}

JNI_FN(void, hllAddAsync)(JNIEnv *env, jclass cls, jlong space, jstring name, jobject keys, jobject offsets, jlong n,
                          jobject done) {
  (void)cls;
  reap(env);
  jname nm;
  if (name_get(env, name, &nm)) return;
  job *j = job_new(env, done, K_BOOL, 0);
  if (!j) {
    name_put(env, &nm);
    return;
  }
  const int rc = rsk_shim_hll_add_async(space, nm.c, direct(env, keys), direct(env, offsets), n, jni_done, j);
  name_put(env, &nm);
  if (rc) job_refused(env, j, rc);
}

JNI_FN(void, hllCountAsync)(JNIEnv *env, jclass cls, jlong space, jstring name, jobject done) {
  (void)cls;
  reap(env);
  jname nm;
  if (name_get(env, name, &nm)) return;
  job *j = job_new(env, done, K_LONG, 0);
  if (!j) {
    name_put(env, &nm);
    return;
  }
  const int rc = rsk_shim_hll_count_async(space, nm.c, jni_done, j);
  name_put(env, &nm);
  if (rc) job_refused(env, j, rc);
}

JNI_FN(void, hllCountWithAsync)(JNIEnv *env, jclass cls, jlong space, jobjectArray names, jobject done) {
  (void)cls;
  reap(env);
  jnames ns;
  if (names_get(env, names, &ns)) {
    names_put(env, &ns);
    return;
  }
  job *j = job_new(env, done, K_LONG, 0);
  const int rc = j ? rsk_shim_hll_count_with_async(space, ns.cs, ns.k, jni_done, j) : RSK_ERR_OUT_OF_MEMORY;
  names_put(env, &ns);
  if (rc && j) job_refused(env, j, rc);
  else if (rc) raise(env, rc);
}

JNI_FN(void, hllMergeWithAsync)(JNIEnv *env, jclass cls, jlong space, jstring dst, jobjectArray srcs, jobject done) {
  (void)cls;
  reap(env);
  jname d;
  if (name_get(env, dst, &d)) return;
  jnames ns;
  if (names_get(env, srcs, &ns)) {
    names_put(env, &ns);
    name_put(env, &d);
    return;
  }
  job *j = job_new(env, done, K_VOID, 0);
  const int rc = j ? rsk_shim_hll_merge_with_async(space, d.c, ns.cs, ns.k, jni_done, j) : RSK_ERR_OUT_OF_MEMORY;
  names_put(env, &ns);
  name_put(env, &d);
  if (rc && j) job_refused(env, j, rc);
  else if (rc) raise(env, rc);
}

/* ---------------------------------------------------------------- Bloom */
/* cfg[0] = size, cfg[1] = hashIterations, cfg[2] = expectedInsertions; fpp[0] = falseProbability */
static void put_config(JNIEnv *env, const rsk_shim_bloom_config *c, jlongArray cfg, jdoubleArray fpp) {
  const jlong v[3] = {(jlong)c->size, (jlong)c->hash_iterations, (jlong)c->expected_insertions};
  const jdouble p = c->false_probability;
  if (cfg) (*env)->SetLongArrayRegion(env, cfg, 0, 3, v);
  if (fpp) (*env)->SetDoubleArrayRegion(env, fpp, 0, 1, &p);
}

JNI_FN(jboolean, bloomTryInit)(JNIEnv *env, jclass cls, jlong space, jstring name, jlong n, jdouble p, jlongArray cfg,
                               jdoubleArray fpp) {
  (void)cls;
  reap(env);
  jname nm;
  if (name_get(env, name, &nm)) return JNI_FALSE;
  int32_t created = 0;
  rsk_shim_bloom_config c;
  const int rc = rsk_shim_bloom_try_init(space, nm.c, n, p, &created, &c);
  name_put(env, &nm);
  if (raise(env, rc)) return JNI_FALSE;
  put_config(env, &c, cfg, fpp);
  return created ? JNI_TRUE : JNI_FALSE;
}

JNI_FN(void, bloomConfig)(JNIEnv *env, jclass cls, jlong space, jstring name, jlongArray cfg, jdoubleArray fpp) {
  (void)cls;
  reap(env);
  jname nm;
  if (name_get(env, name, &nm)) return;
  rsk_shim_bloom_config c;
  const int rc = rsk_shim_bloom_get_config(space, nm.c, &c);
  name_put(env, &nm);
  if (!raise(env, rc)) put_config(env, &c, cfg, fpp);
}

static jbooleanArray bloom_batch(JNIEnv *env, jlong space, jstring name, jlong size, jint k, jobject keys,
                                 jobject offsets, jlong n, int add) {
  uint8_t *r = reply_buf(env, n);
  if (!r) return NULL;
  jname nm;
  if (name_get(env, name, &nm)) {
    free(r);
    return NULL;
  }
  const int rc = add ? rsk_shim_bloom_add(space, nm.c, size, k, direct(env, keys), direct(env, offsets), n, r, n)
                     : rsk_shim_bloom_contains(space, nm.c, size, k, direct(env, keys), direct(env, offsets), n, r, n);
  name_put(env, &nm);
  jbooleanArray arr = raise(env, rc) ? NULL : replies_array(env, r, n);
  free(r);
  return arr;
}

JNI_FN(jbooleanArray, bloomAdd)(JNIEnv *env, jclass cls, jlong space, jstring name, jlong size, jint k, jobject keys,
                                jobject offsets, jlong n) {
  (void)cls;
  reap(env);
  return bloom_batch(env, space, name, size, k, keys, offsets, n, 1);
}

JNI_FN(jbooleanArray, bloomContains)(JNIEnv *env, jclass cls, jlong space, jstring name, jlong size, jint k,
                                     jobject keys, jobject offsets, jlong n) {
  (void)cls;
  reap(env);
  return bloom_batch(env, space, name, size, k, keys, offsets, n, 0);
}

JNI_FN(jint, bloomCount)(JNIEnv *env, jclass cls, jlong space, jstring name) {
  (void)cls;
  reap(env);
  jname nm;
  if (name_get(env, name, &nm)) return 0;
  int32_t v = 0;
  const int rc = rsk_shim_bloom_count(space, nm.c, &v);
  name_put(env, &nm);
  return raise(env, rc) ? 0 : (jint)v;
}

static void bloom_async(JNIEnv *env, jlong space, jstring name, jlong size, jint k, jobject keys, jobject offsets,
                        jlong n, jobject done, int add) {
  if (n < 0 || n > 0x7fffffff) {
    throw_iae(env, "batch larger than 2^31 - 1 elements");
    return;
  }
  jname nm;
  if (name_get(env, name, &nm)) return;
  job *j = job_new(env, done, K_ARRAY, n);
  if (!j) {
    name_put(env, &nm);
    return;
  }
  const int rc = add ? rsk_shim_bloom_add_async(space, nm.c, size, k, direct(env, keys), direct(env, offsets), n,
                                                j->out, n, jni_done, j)
                     : rsk_shim_bloom_contains_async(space, nm.c, size, k, direct(env, keys), direct(env, offsets),
                                                     n, j->out, n, jni_done, j);
  name_put(env, &nm);
  if (rc) job_refused(env, j, rc);
}

JNI_FN(void, bloomAddAsync)(JNIEnv *env, jclass cls, jlong space, jstring name, jlong size, jint k, jobject keys,
                            jobject offsets, jlong n, jobject done) {
  (void)cls;
  reap(env);
  bloom_async(env, space, name, size, k, keys, offsets, n, done, 1);
}

JNI_FN(void, bloomContainsAsync)(JNIEnv *env, jclass cls, jlong space, jstring name, jlong size, jint k, jobject keys,
                                 jobject offsets, jlong n, jobject done) {
  (void)cls;
  reap(env);
  bloom_async(env, space, name, size, k, keys, offsets, n, done, 0);
}

/* -------------------------------------------------------------- RBitSet */
/* long[] -> C copy (NULL with a pending exception on failure). */
static int64_t *long_array(JNIEnv *env, jlongArray a, jsize *n) {
  *n = a ? (*env)->GetArrayLength(env, a) : 0;
  if (!a) {
    throw_iae(env, "bit indexes are null");
    return NULL;
  }
  int64_t *v = malloc(sizeof(int64_t) * (size_t)(*n > 0 ? *n : 1));
  if (!v) {
    jclass c = (*env)->FindClass(env, "java/lang/OutOfMemoryError");
    if (c) (*env)->ThrowNew(env, c, "bit indexes");
    return NULL;
  }
  if (*n) (*env)->GetLongArrayRegion(env, a, 0, *n, (jlong *)v);
  return v;
}

JNI_FN(jlong, bitsetStrlen)(JNIEnv *env, jclass cls, jlong space, jstring name) {
  (void)cls;
  reap(env);
  jname nm;
  if (name_get(env, name, &nm)) return 0;
  int64_t v = 0;
  const int rc = rsk_shim_bitset_strlen(space, nm.c, &v);
  name_put(env, &nm);
  return raise(env, rc) ? 0 : (jlong)v;
}

JNI_FN(jbyteArray, bitsetGet)(JNIEnv *env, jclass cls, jlong space, jstring name) {
  (void)cls;
  reap(env);
  jname nm;
  if (name_get(env, name, &nm)) return NULL;
  uint8_t *bytes = NULL;
  int64_t len = -1;
  const int rc = rsk_shim_bitset_get_bytes(space, nm.c, &bytes, &len);
  name_put(env, &nm);
  jbyteArray arr = NULL;
  if (!raise(env, rc) && len >= 0) { /* len -1: GET nil -> null */
    arr = (*env)->NewByteArray(env, (jsize)len);
    if (arr && len) (*env)->SetByteArrayRegion(env, arr, 0, (jsize)len, (const jbyte *)bytes);
  }
  rsk_shim_free(bytes);
  return arr;
}

JNI_FN(jbooleanArray, bitsetGetBits)(JNIEnv *env, jclass cls, jlong space, jstring name, jlongArray indexes) {
  (void)cls;
  reap(env);
  jsize n = 0;
  int64_t *offs = long_array(env, indexes, &n);
  if (!offs) return NULL;
  uint8_t *r = reply_buf(env, n);
  jname nm;
  jbooleanArray arr = NULL;
  if (r && !name_get(env, name, &nm)) {
    const int rc = rsk_shim_bitset_getbits(space, nm.c, offs, n, r, n);
    name_put(env, &nm);
    if (!raise(env, rc)) arr = replies_array(env, r, n);
  }
  free(r);
  free(offs);
  return arr;
}

JNI_FN(void, bitsetSetBits)(JNIEnv *env, jclass cls, jlong space, jstring name, jlongArray indexes,
                            jboolean value) {
  (void)cls;
  reap(env);
  jsize n = 0;
  int64_t *offs = long_array(env, indexes, &n);
  if (!offs) return;
  jname nm;
  if (!name_get(env, name, &nm)) {
    const int rc = rsk_shim_bitset_setbits(space, nm.c, offs, n, value ? 1 : 0);
    name_put(env, &nm);
    raise(env, rc);
  }
  free(offs);
}

JNI_FN(void, bitsetSetRange)(JNIEnv *env, jclass cls, jlong space, jstring name, jlong from, jlong to,
                             jboolean value) {
  (void)cls;
  reap(env);
  jname nm;
  if (name_get(env, name, &nm)) return;
  const int rc = rsk_shim_bitset_set_range(space, nm.c, from, to, value ? 1 : 0);
  name_put(env, &nm);
  raise(env, rc);
}

JNI_FN(jlong, bitsetCardinality)(JNIEnv *env, jclass cls, jlong space, jstring name) {
  (void)cls;
  reap(env);
  jname nm;
  if (name_get(env, name, &nm)) return 0;
  int64_t v = 0;
  const int rc = rsk_shim_bitset_cardinality(space, nm.c, &v);
  name_put(env, &nm);
  return raise(env, rc) ? 0 : (jlong)v;
}

JNI_FN(jlong, bitsetLength)(JNIEnv *env, jclass cls, jlong space, jstring name) {
  (void)cls;
  reap(env);
  jname nm;
  if (name_get(env, name, &nm)) return 0;
  int64_t v = 0;
  const int rc = rsk_shim_bitset_length(space, nm.c, &v);
  name_put(env, &nm);
  return raise(env, rc) ? 0 : (jlong)v;
}

JNI_FN(void, bitsetSet)(JNIEnv *env, jclass cls, jlong space, jstring name, jbyteArray bytes) {
  (void)cls;
  reap(env);
  if (!bytes) {
    throw_iae(env, "bytes is null");
    return;
  }
  const jsize n = (*env)->GetArrayLength(env, bytes);
  uint8_t *v = malloc((size_t)(n > 0 ? n : 1));
  if (!v) {
    jclass c = (*env)->FindClass(env, "java/lang/OutOfMemoryError");
    if (c) (*env)->ThrowNew(env, c, "bytes");
    return;
  }
  if (n) (*env)->GetByteArrayRegion(env, bytes, 0, n, (jbyte *)v);
  jname nm;
  if (!name_get(env, name, &nm)) {
    const int rc = rsk_shim_bitset_set_bytes(space, nm.c, v, n);
    name_put(env, &nm);
    raise(env, rc);
  }
  free(v);
}

JNI_FN(jboolean, bitsetClear)(JNIEnv *env, jclass cls, jlong space, jstring name) {
  (void)cls;
  reap(env);
  jname nm;
  if (name_get(env, name, &nm)) return JNI_FALSE;
  int32_t d = 0;
  const int rc = rsk_shim_bitset_clear(space, nm.c, &d);
  name_put(env, &nm);
  return raise(env, rc) ? JNI_FALSE : (d ? JNI_TRUE : JNI_FALSE);
}

JNI_FN(void, bitsetOp)(JNIEnv *env, jclass cls, jlong space, jstring name, jint op, jobjectArray others) {
  (void)cls;
  reap(env);
  jname nm;
  if (name_get(env, name, &nm)) return;
  jnames ns;
  if (names_get(env, others, &ns)) {
    names_put(env, &ns);
    name_put(env, &nm);
    return;
  }
  const int rc = rsk_shim_bitset_op(space, nm.c, op, ns.cs, ns.k);
  names_put(env, &ns);
  name_put(env, &nm);
  raise(env, rc);
}

/*
 * rsketch_jni.c -- JNI glue of org.redisson.gpu.RSketchNative
 * (jni/java/org/redisson/gpu/RSketchNative.java) over rsketch_shim.c.
 *
 * Needs a JDK's jni.h, which this image lacks: it is source here and is built
 * where JAVA_HOME exists (make -C jni jni).  Every method follows one pattern:
 * fetch direct-buffer addresses and capacities, call the shim, throw
 * rsk_shim_exception_class(rc) with rsk_shim_last_error() on failure.  The
 * shim (all checks, all conversions) is what tests/c/shim_caller.c runs on
 * the GPU.
 */
#include <jni.h>
#include <stdlib.h>

#include "rsketch_shim.h"

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

#define JNI_FN(ret, name) JNIEXPORT ret JNICALL Java_org_redisson_gpu_RSketchNative_##name

JNI_FN(jlong, init)(JNIEnv *env, jclass cls, jint device) {
  (void)cls;
  int64_t ctx = 0;
  return raise(env, rsk_shim_init(device, &ctx)) ? 0 : (jlong)ctx;
}

JNI_FN(void, shutdown)(JNIEnv *env, jclass cls, jlong ctx) {
  (void)cls;
  raise(env, rsk_shim_shutdown(ctx));
}

JNI_FN(jlong, hllCreate)(JNIEnv *env, jclass cls, jlong ctx, jlong n) {
  (void)cls;
  int64_t h = 0;
  return raise(env, rsk_shim_hll_create(ctx, n, &h)) ? 0 : (jlong)h;
}

JNI_FN(void, hllDestroy)(JNIEnv *env, jclass cls, jlong hll) {
  (void)cls;
  raise(env, rsk_shim_hll_destroy(hll));
}

JNI_FN(jboolean, hllAdd)(JNIEnv *env, jclass cls, jlong hll, jlong id, jobject keys, jobject offsets, jlong n) {
  (void)cls;
  uint8_t changed = 0;
  if (raise(env, rsk_shim_hll_add(hll, id, direct(env, keys), direct(env, offsets), n, &changed))) return JNI_FALSE;
  return changed ? JNI_TRUE : JNI_FALSE;
}

/* boolean[] replies: jboolean is an unsigned byte, so the library writes the
 * replies straight into the array's elements. */
JNI_FN(jbooleanArray, hllAddEach)(JNIEnv *env, jclass cls, jlong hll, jlong id, jobject keys, jobject offsets,
                                  jlong n) {
  (void)cls;
  if (n < 0 || n > 0x7fffffff) {
    raise(env, RSK_ERR_INVALID_ARG);
    return NULL;
  }
  jbooleanArray arr = (*env)->NewBooleanArray(env, (jsize)n);
  if (!arr) return NULL;
  jboolean *r = (*env)->GetBooleanArrayElements(env, arr, NULL);
  int rc = rsk_shim_hll_add_each(hll, id, direct(env, keys), direct(env, offsets), n, (uint8_t *)r, n);
  (*env)->ReleaseBooleanArrayElements(env, arr, r, rc ? JNI_ABORT : 0);
  return raise(env, rc) ? NULL : arr;
}

JNI_FN(jlong, hllCount)(JNIEnv *env, jclass cls, jlong hll, jlong id) {
  (void)cls;
  int64_t v = 0;
  return raise(env, rsk_shim_hll_count(hll, id, &v)) ? 0 : (jlong)v;
}

JNI_FN(jlong, hllCountUnion)(JNIEnv *env, jclass cls, jlongArray hlls, jlongArray ids) {
  (void)cls;
  const jsize k = (*env)->GetArrayLength(env, hlls);
  if (k != (*env)->GetArrayLength(env, ids)) {
    raise(env, RSK_ERR_INVALID_ARG);
    return 0;
  }
  jlong *h = (*env)->GetLongArrayElements(env, hlls, NULL);
  jlong *i = (*env)->GetLongArrayElements(env, ids, NULL);
  int64_t v = 0;
  int rc = rsk_shim_hll_count_union((const int64_t *)h, (const int64_t *)i, (int32_t)k, &v);
  (*env)->ReleaseLongArrayElements(env, ids, i, JNI_ABORT);
  (*env)->ReleaseLongArrayElements(env, hlls, h, JNI_ABORT);
  return raise(env, rc) ? 0 : (jlong)v;
}

JNI_FN(void, hllMerge)(JNIEnv *env, jclass cls, jlong dst, jlong dstId, jlongArray srcs, jlongArray srcIds) {
  (void)cls;
  const jsize k = (*env)->GetArrayLength(env, srcs);
  if (k != (*env)->GetArrayLength(env, srcIds)) {
    raise(env, RSK_ERR_INVALID_ARG);
    return;
  }
  jlong *h = (*env)->GetLongArrayElements(env, srcs, NULL);
  jlong *i = (*env)->GetLongArrayElements(env, srcIds, NULL);
  int rc = rsk_shim_hll_merge(dst, dstId, (const int64_t *)h, (const int64_t *)i, (int32_t)k);
  (*env)->ReleaseLongArrayElements(env, srcIds, i, JNI_ABORT);
  (*env)->ReleaseLongArrayElements(env, srcs, h, JNI_ABORT);
  raise(env, rc);
}

JNI_FN(void, hllDelete)(JNIEnv *env, jclass cls, jlong hll, jlong id) {
  (void)cls;
  raise(env, rsk_shim_hll_delete(hll, id));
}

/* {size, k} */
JNI_FN(jlongArray, bloomParams)(JNIEnv *env, jclass cls, jlong n, jdouble p, jboolean extended) {
  (void)cls;
  int64_t size = 0;
  int32_t k = 0;
  if (raise(env, rsk_shim_bloom_params(n, p, extended ? 1 : 0, &size, &k))) return NULL;
  jlongArray arr = (*env)->NewLongArray(env, 2);
  if (!arr) return NULL;
  const jlong v[2] = {(jlong)size, (jlong)k};
  (*env)->SetLongArrayRegion(env, arr, 0, 2, v);
  return arr;
}

JNI_FN(jlong, bloomCreate)(JNIEnv *env, jclass cls, jlong ctx, jlong size, jint k) {
  (void)cls;
  int64_t b = 0;
  return raise(env, rsk_shim_bloom_create(ctx, size, k, &b)) ? 0 : (jlong)b;
}

JNI_FN(void, bloomDestroy)(JNIEnv *env, jclass cls, jlong bloom) {
  (void)cls;
  raise(env, rsk_shim_bloom_destroy(bloom));
}

static jbooleanArray bloom_batch(JNIEnv *env, jlong bloom, jobject keys, jobject offsets, jlong n, int add) {
  if (n < 0 || n > 0x7fffffff) {
    raise(env, RSK_ERR_INVALID_ARG);
    return NULL;
  }
  jbooleanArray arr = (*env)->NewBooleanArray(env, (jsize)n);
  if (!arr) return NULL;
  jboolean *r = (*env)->GetBooleanArrayElements(env, arr, NULL);
  int rc = add ? rsk_shim_bloom_add(bloom, direct(env, keys), direct(env, offsets), n, (uint8_t *)r, n)
               : rsk_shim_bloom_contains(bloom, direct(env, keys), direct(env, offsets), n, (uint8_t *)r, n);
  (*env)->ReleaseBooleanArrayElements(env, arr, r, rc ? JNI_ABORT : 0);
  return raise(env, rc) ? NULL : arr;
}

JNI_FN(jbooleanArray, bloomAdd)(JNIEnv *env, jclass cls, jlong bloom, jobject keys, jobject offsets, jlong n) {
  (void)cls;
  return bloom_batch(env, bloom, keys, offsets, n, 1);
}

JNI_FN(jbooleanArray, bloomContains)(JNIEnv *env, jclass cls, jlong bloom, jobject keys, jobject offsets, jlong n) {
  (void)cls;
  return bloom_batch(env, bloom, keys, offsets, n, 0);
}

JNI_FN(jint, bloomCount)(JNIEnv *env, jclass cls, jlong bloom) {
  (void)cls;
  int32_t v = 0;
  return raise(env, rsk_shim_bloom_count(bloom, &v)) ? 0 : (jint)v;
}

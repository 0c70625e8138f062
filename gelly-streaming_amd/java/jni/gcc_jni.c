/* NOT COMPILED IN THIS IMAGE (no JDK / jni.h): the JNI glue of the reference-side bridge
 * (gelly-streaming_amd/java/README.md). Build: cc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux
 *   -I../../../include gcc_jni.c -L../../lib -lgelly_cc -o libgelly_cc_jni.so
 * Each function forwards to one C-ABI call of include/gelly_cc.h; a negative status becomes a GccException carrying
 * gcc_last_error(). Handles travel as jlong. */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

#include "gelly_cc.h"

#define H(x) ((gcc_forest*)(intptr_t)(x))

static int fail(JNIEnv* env, int rc) {
    if (rc >= 0) return 0;
    jclass k = (*env)->FindClass(env, "org/apache/flink/graph/streaming/gpu/GccException");
    jmethodID ctor = (*env)->GetMethodID(env, k, "<init>", "(ILjava/lang/String;)V");
    jstring msg = (*env)->NewStringUTF(env, gcc_last_error());
    (*env)->Throw(env, (jthrowable)(*env)->NewObject(env, k, ctor, (jint)rc, msg));
    return 1;
}

#define FN(ret, name) JNIEXPORT ret JNICALL Java_org_apache_flink_graph_streaming_gpu_Gcc_##name

FN(jlong, create)(JNIEnv* env, jclass c, jint device, jint cap) {
    gcc_forest* h = 0;
    if (fail(env, gcc_forest_create(device, (uint32_t)cap, &h))) return 0;
    return (jlong)(intptr_t)h;
}

FN(void, destroy)(JNIEnv* env, jclass c, jlong h) { (void)gcc_forest_destroy(H(h)); }

/* the library-owned pinned staging slot, zero-copy: Java writes (u32, u32) pairs straight into it */
FN(jobject, staging)(JNIEnv* env, jclass c, jlong h) {
    uint32_t* p = 0;
    uint64_t cap = 0;
    if (fail(env, gcc_forest_staging(H(h), &p, &cap))) return 0;
    return (*env)->NewDirectByteBuffer(env, p, (jlong)(cap * 2 * sizeof(uint32_t)));
}

FN(void, submit)(JNIEnv* env, jclass c, jlong h, jlong n) { fail(env, gcc_forest_submit(H(h), (uint64_t)n)); }
FN(void, sync)(JNIEnv* env, jclass c, jlong h) { fail(env, gcc_forest_sync(H(h))); }

FN(jlong, size)(JNIEnv* env, jclass c, jlong h) {
    uint64_t n = 0;
    if (fail(env, gcc_forest_size(H(h), &n))) return 0;
    return (jlong)n;
}

FN(void, labels)(JNIEnv* env, jclass c, jlong h, jintArray out) {
    const jsize n = (*env)->GetArrayLength(env, out);
    jint* p = (*env)->GetIntArrayElements(env, out, 0);
    const int rc = gcc_forest_labels(H(h), (uint32_t*)p, (uint32_t)n);
    (*env)->ReleaseIntArrayElements(env, out, p, rc < 0 ? JNI_ABORT : 0);
    fail(env, rc);
}

FN(void, merge)(JNIEnv* env, jclass c, jlong into, jlong from) { fail(env, gcc_forest_merge(H(into), H(from))); }
FN(void, reset)(JNIEnv* env, jclass c, jlong h) { fail(env, gcc_forest_reset(H(h))); }

FN(jbyteArray, serialize)(JNIEnv* env, jclass c, jlong h) {
    uint64_t n = 0, w = 0;
    if (fail(env, gcc_forest_serialized_size(H(h), &n))) return 0;
    void* buf = malloc((size_t)n);
    if (!buf) {
        fail(env, GCC_E_OOM);
        return 0;
    }
    const int rc = gcc_forest_serialize(H(h), buf, n, &w);
    jbyteArray out = 0;
    if (rc >= 0) {
        out = (*env)->NewByteArray(env, (jsize)w);
        (*env)->SetByteArrayRegion(env, out, 0, (jsize)w, (const jbyte*)buf);
    }
    free(buf);
    fail(env, rc);
    return out;
}

FN(void, deserialize)(JNIEnv* env, jclass c, jlong h, jbyteArray data) {
    const jsize n = (*env)->GetArrayLength(env, data);
    jbyte* p = (*env)->GetByteArrayElements(env, data, 0);
    const int rc = gcc_forest_deserialize(H(h), p, (uint64_t)n);
    (*env)->ReleaseByteArrayElements(env, data, p, JNI_ABORT);
    fail(env, rc);
}

/* ---- Long vertex ids (DisjointSet<Long> takes any Long, …/summaries/DisjointSet.java:30-34): the id dictionary of
 * include/gelly_cc.h, gcc_idmap_* ---- */
#define M(x) ((gcc_idmap*)(intptr_t)(x))

FN(jlong, idmapCreate)(JNIEnv* env, jclass c, jint capacity) {
    gcc_idmap* m = 0;
    if (fail(env, gcc_idmap_create((uint32_t)capacity, &m))) return 0;
    return (jlong)(intptr_t)m;
}

FN(void, idmapDestroy)(JNIEnv* env, jclass c, jlong m) { (void)gcc_idmap_destroy(M(m)); }

/* nPairs (Long src, Long dst) pairs: map every id to its dense id straight into the pinned staging slot, then
 * submit the slot (the same call sequence as a direct-id batch: staging -> fill -> submit) */
FN(void, submitLong)(JNIEnv* env, jclass c, jlong h, jlong m, jlongArray pairs, jint nPairs) {
    uint32_t* slot = 0;
    uint64_t cap = 0;
    if (fail(env, gcc_forest_staging(H(h), &slot, &cap))) return;
    if ((uint64_t)nPairs > cap) {
        fail(env, GCC_E_INVALID);
        return;
    }
    jlong* p = (*env)->GetLongArrayElements(env, pairs, 0);
    int rc = gcc_idmap_map(M(m), (const int64_t*)p, 2 * (uint64_t)nPairs, slot);
    (*env)->ReleaseLongArrayElements(env, pairs, p, JNI_ABORT);
    if (fail(env, rc)) return;
    fail(env, gcc_forest_submit(H(h), (uint64_t)nPairs));
}

/* dense id of `id`, or -1 (GCC_UNSEEN) if it was never mapped */
FN(jint, idmapLookup)(JNIEnv* env, jclass c, jlong m, jlong id) {
    uint32_t d = GCC_UNSEEN;
    if (fail(env, gcc_idmap_lookup(M(m), (int64_t)id, &d))) return -1;
    return (jint)d;
}

/* out[d] = original id of dense id d, for every mapped id */
FN(jlongArray, idmapIds)(JNIEnv* env, jclass c, jlong m) {
    uint64_t n = 0;
    if (fail(env, gcc_idmap_size(M(m), &n))) return 0;
    jlongArray out = (*env)->NewLongArray(env, (jsize)n);
    jlong* p = (*env)->GetLongArrayElements(env, out, 0);
    const int rc = gcc_idmap_ids(M(m), (int64_t*)p, n);
    (*env)->ReleaseLongArrayElements(env, out, p, rc < 0 ? JNI_ABORT : 0);
    fail(env, rc);
    return out;
}

/* per dense id: the minimum ORIGINAL id of its component (the reference's canonical form in signed Long order) */
FN(jlongArray, canonical)(JNIEnv* env, jclass c, jlong h, jlong m) {
    uint64_t n = 0;
    if (fail(env, gcc_idmap_size(M(m), &n))) return 0;
    uint32_t* lab = (uint32_t*)malloc((size_t)(n ? n : 1) * sizeof(uint32_t));
    if (!lab) {
        fail(env, GCC_E_OOM);
        return 0;
    }
    int rc = gcc_forest_labels(H(h), lab, (uint32_t)n);
    jlongArray out = 0;
    if (rc >= 0) {
        out = (*env)->NewLongArray(env, (jsize)n);
        jlong* p = (*env)->GetLongArrayElements(env, out, 0);
        rc = gcc_idmap_canonical(M(m), lab, n, (int64_t*)p, INT64_MIN);
        (*env)->ReleaseLongArrayElements(env, out, p, rc < 0 ? JNI_ABORT : 0);
    }
    free(lab);
    fail(env, rc);
    return out;
}

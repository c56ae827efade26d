/*
 * mock_jni.c — TEST INFRASTRUCTURE: a minimal mock JVM behind the JNI function table of
 * tests/jni/jni.h, so that jni/omr_jni.c (the product JNI shim) runs under pytest without a JDK.
 *
 * Objects are plain heap records (byte / int / double / object arrays, strings, classes,
 * throwables).  Beyond serving the calls, the mock checks the rules the JNI specification puts on
 * native code and counts every breach, which the tests assert to be zero:
 *   - no JNI call other than the critical-region pair while a critical array is held;
 *   - only the exception-safe calls while an exception is pending;
 *   - no null or wrongly typed array handed to an array function;
 *   - array regions inside their array (a breach throws ArrayIndexOutOfBoundsException, as the JVM);
 *   - local references: created minus deleted stays bounded (a leak in a loop shows up here).
 * Test-side helpers (mock_*) build arrays from Python, read results and the pending exception.
 */
#include "jni.h"

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { K_CLASS = 1, K_STRING, K_BYTES, K_INTS, K_DOUBLES, K_OBJECTS, K_THROWABLE };

typedef struct MObj {
    int kind;
    int32_t len;          /* elements (arrays), bytes (string) */
    void* data;
    char name[128];       /* class name / throwable class */
    int32_t status;       /* OmrException status */
    char msg[512];
    struct MObj* next;    /* every object, for mock_reset */
} MObj;

struct _jmethodID { const char* sig; };
static struct _jmethodID kOmrExceptionCtor = {"(ILjava/lang/String;)V"};

static MObj* g_all = NULL;
static MObj* g_pending = NULL;
static int64_t g_local_live = 0, g_local_max = 0, g_crit = 0;
static int64_t g_crit_violations = 0, g_exc_violations = 0, g_arg_violations = 0, g_calls = 0;

static MObj* mk(int kind, int32_t len, size_t elem) {
    MObj* o = (MObj*)calloc(1, sizeof(MObj));
    o->kind = kind;
    o->len = len;
    if (elem) o->data = calloc(len > 0 ? (size_t)len : 1, elem);
    o->next = g_all;
    g_all = o;
    return o;
}

static void local_ref(void) {
    if (++g_local_live > g_local_max) g_local_max = g_local_live;
}

/* Call-site rules: `crit_ok` calls may run inside a critical region, `exc_ok` with an exception
 * pending (JNI spec: ExceptionOccurred/Describe/Clear/Check, the Release* family, DeleteLocalRef). */
static void enter(int crit_ok, int exc_ok) {
    ++g_calls;
    if (g_crit > 0 && !crit_ok) ++g_crit_violations;
    if (g_pending && !exc_ok) ++g_exc_violations;
}

static void throw_named(const char* cls, const char* msg) {
    MObj* t = mk(K_THROWABLE, 0, 0);
    snprintf(t->name, sizeof t->name, "%s", cls);
    snprintf(t->msg, sizeof t->msg, "%s", msg);
    t->status = -1;
    g_pending = t;
}

static MObj* arr(jobject a, int kind) {
    MObj* o = (MObj*)a;
    if (!o || o->kind != kind) {
        ++g_arg_violations;
        return NULL;
    }
    return o;
}

static int region_ok(MObj* o, jsize start, jsize len) {
    if (start < 0 || len < 0 || (int64_t)start + len > o->len) {
        throw_named("java/lang/ArrayIndexOutOfBoundsException", "region outside the array");
        return 0;
    }
    return 1;
}

/* ---- the JNI functions the shim calls ----------------------------------------------------- */
static jint JNICALL m_GetVersion(JNIEnv* env) { enter(0, 0); return 0x00010008; }

static jclass JNICALL m_FindClass(JNIEnv* env, const char* name) {
    enter(0, 0);
    if (strcmp(name, "com/glencoesoftware/omero/ms/image/region/gpu/OmrException") != 0) {
        throw_named("java/lang/NoClassDefFoundError", name);
        return NULL;
    }
    MObj* c = mk(K_CLASS, 0, 0);
    snprintf(c->name, sizeof c->name, "%s", name);
    local_ref();
    return (jclass)c;
}

static jint JNICALL m_Throw(JNIEnv* env, jthrowable t) {
    enter(0, 0);
    MObj* o = (MObj*)t;
    if (!o || o->kind != K_THROWABLE) { ++g_arg_violations; return -1; }
    g_pending = o;
    return 0;
}

static jint JNICALL m_ThrowNew(JNIEnv* env, jclass c, const char* msg) {
    enter(0, 0);
    throw_named(c ? ((MObj*)c)->name : "?", msg ? msg : "");
    return 0;
}

static jthrowable JNICALL m_ExceptionOccurred(JNIEnv* env) { enter(1, 1); return (jthrowable)g_pending; }
static void JNICALL m_ExceptionClear(JNIEnv* env) { enter(1, 1); g_pending = NULL; }
static jboolean JNICALL m_ExceptionCheck(JNIEnv* env) { enter(1, 1); return g_pending != NULL; }

static void JNICALL m_DeleteLocalRef(JNIEnv* env, jobject o) {
    enter(0, 1);
    if (o) --g_local_live;
}

static jmethodID JNICALL m_GetMethodID(JNIEnv* env, jclass c, const char* name, const char* sig) {
    enter(0, 0);
    MObj* k = (MObj*)c;
    if (!k || k->kind != K_CLASS) { ++g_arg_violations; return NULL; }
    if (strcmp(name, "<init>") || strcmp(sig, kOmrExceptionCtor.sig)) {
        throw_named("java/lang/NoSuchMethodError", name);
        return NULL;
    }
    return &kOmrExceptionCtor;
}

static jobject JNICALL m_NewObject(JNIEnv* env, jclass c, jmethodID m, ...) {
    enter(0, 0);
    if (!c || m != &kOmrExceptionCtor) { ++g_arg_violations; return NULL; }
    va_list ap;
    va_start(ap, m);
    const jint status = va_arg(ap, jint);
    MObj* s = (MObj*)va_arg(ap, jstring);
    va_end(ap);
    MObj* t = mk(K_THROWABLE, 0, 0);
    snprintf(t->name, sizeof t->name, "%s", ((MObj*)c)->name);
    t->status = status;
    if (s && s->kind == K_STRING) snprintf(t->msg, sizeof t->msg, "%s", (const char*)s->data);
    local_ref();
    return (jobject)t;
}

static jstring JNICALL m_NewStringUTF(JNIEnv* env, const char* utf) {
    enter(0, 0);
    const size_t n = strlen(utf);
    MObj* s = mk(K_STRING, (int32_t)n, 1);
    free(s->data);
    s->data = malloc(n + 1);
    memcpy(s->data, utf, n + 1);
    local_ref();
    return (jstring)s;
}

static const char* JNICALL m_GetStringUTFChars(JNIEnv* env, jstring s, jboolean* is_copy) {
    enter(0, 0);
    MObj* o = arr(s, K_STRING);
    if (is_copy) *is_copy = JNI_FALSE;
    return o ? (const char*)o->data : NULL;
}

static void JNICALL m_ReleaseStringUTFChars(JNIEnv* env, jstring s, const char* p) { enter(0, 1); }

static jsize JNICALL m_GetArrayLength(JNIEnv* env, jarray a) {
    enter(0, 0);
    MObj* o = (MObj*)a;
    if (!o || o->kind < K_BYTES || o->kind > K_OBJECTS) { ++g_arg_violations; return 0; }
    return o->len;
}

static jobject JNICALL m_GetObjectArrayElement(JNIEnv* env, jobjectArray a, jsize i) {
    enter(0, 0);
    MObj* o = arr(a, K_OBJECTS);
    if (!o) return NULL;
    if (i < 0 || i >= o->len) {
        throw_named("java/lang/ArrayIndexOutOfBoundsException", "element");
        return NULL;
    }
    jobject e = ((jobject*)o->data)[i];
    if (e) local_ref();
    return e;
}

static jbyteArray JNICALL m_NewByteArray(JNIEnv* env, jsize len) {
    enter(0, 0);
    if (len < 0) { ++g_arg_violations; return NULL; }
    local_ref();
    return (jbyteArray)mk(K_BYTES, len, 1);
}

#define REGION(NAME, KIND, T, DIR)                                                                  \
    static void JNICALL m_##NAME(JNIEnv* env, jarray a, jsize start, jsize len, DIR T* buf) {         \
        enter(0, 0);                                                                                \
        MObj* o = arr(a, KIND);                                                                     \
        if (!o || !region_ok(o, start, len)) return;                                                \
        if (len && !buf) { ++g_arg_violations; return; }                                            \
        REGION_COPY_##DIR(o, T, start, len, buf);                                                   \
    }
#define REGION_COPY_(o, T, start, len, buf) memcpy((buf), (T*)(o)->data + (start), sizeof(T) * (size_t)(len))
#define REGION_COPY_const(o, T, start, len, buf) memcpy((T*)(o)->data + (start), (buf), sizeof(T) * (size_t)(len))
REGION(GetByteArrayRegion, K_BYTES, jbyte, )
REGION(GetIntArrayRegion, K_INTS, jint, )
REGION(GetDoubleArrayRegion, K_DOUBLES, jdouble, )
REGION(SetByteArrayRegion, K_BYTES, jbyte, const)
REGION(SetIntArrayRegion, K_INTS, jint, const)

static void* JNICALL m_GetPrimitiveArrayCritical(JNIEnv* env, jarray a, jboolean* is_copy) {
    enter(1, 0);
    MObj* o = (MObj*)a;
    if (!o || o->kind < K_BYTES || o->kind > K_DOUBLES) { ++g_arg_violations; return NULL; }
    ++g_crit;
    if (is_copy) *is_copy = JNI_FALSE;
    return o->data;
}

static void JNICALL m_ReleasePrimitiveArrayCritical(JNIEnv* env, jarray a, void* p, jint mode) {
    enter(1, 1);
    --g_crit;
}

static struct JNINativeInterface_ g_table;
static const struct JNINativeInterface_* g_env = &g_table;

static void init_table(void) {
    static int done = 0;
    if (done) return;
    done = 1;
    memset(&g_table, 0, sizeof g_table);
    g_table.GetVersion = m_GetVersion;
    g_table.FindClass = m_FindClass;
    g_table.Throw = m_Throw;
    g_table.ThrowNew = m_ThrowNew;
    g_table.ExceptionOccurred = m_ExceptionOccurred;
    g_table.ExceptionClear = m_ExceptionClear;
    g_table.ExceptionCheck = m_ExceptionCheck;
    g_table.DeleteLocalRef = m_DeleteLocalRef;
    g_table.GetMethodID = m_GetMethodID;
    g_table.NewObject = m_NewObject;
    g_table.NewStringUTF = m_NewStringUTF;
    g_table.GetStringUTFChars = m_GetStringUTFChars;
    g_table.ReleaseStringUTFChars = m_ReleaseStringUTFChars;
    g_table.GetArrayLength = m_GetArrayLength;
    g_table.GetObjectArrayElement = m_GetObjectArrayElement;
    g_table.NewByteArray = m_NewByteArray;
    g_table.GetByteArrayRegion = (void (JNICALL*)(JNIEnv*, jbyteArray, jsize, jsize, jbyte*))m_GetByteArrayRegion;
    g_table.GetIntArrayRegion = (void (JNICALL*)(JNIEnv*, jintArray, jsize, jsize, jint*))m_GetIntArrayRegion;
    g_table.GetDoubleArrayRegion =
        (void (JNICALL*)(JNIEnv*, jdoubleArray, jsize, jsize, jdouble*))m_GetDoubleArrayRegion;
    g_table.SetByteArrayRegion =
        (void (JNICALL*)(JNIEnv*, jbyteArray, jsize, jsize, const jbyte*))m_SetByteArrayRegion;
    g_table.SetIntArrayRegion = (void (JNICALL*)(JNIEnv*, jintArray, jsize, jsize, const jint*))m_SetIntArrayRegion;
    g_table.GetPrimitiveArrayCritical = m_GetPrimitiveArrayCritical;
    g_table.ReleasePrimitiveArrayCritical = m_ReleasePrimitiveArrayCritical;
}

/* ---- test-side helpers --------------------------------------------------------------------- */
JNIEnv* mock_env(void) {
    init_table();
    return (JNIEnv*)&g_env;
}

static jobject mk_array(int kind, const void* data, int32_t len, size_t elem) {
    MObj* o = mk(kind, len, elem);
    if (data && len > 0) memcpy(o->data, data, elem * (size_t)len);
    return (jobject)o;
}

jobject mock_bytes(const void* data, int32_t len) { return mk_array(K_BYTES, data, len, 1); }
jobject mock_ints(const void* data, int32_t len) { return mk_array(K_INTS, data, len, 4); }
jobject mock_doubles(const void* data, int32_t len) { return mk_array(K_DOUBLES, data, len, 8); }
jobject mock_objects(int32_t len) { return mk_array(K_OBJECTS, NULL, len, sizeof(jobject)); }
void mock_set(jobject a, int32_t i, jobject v) { ((jobject*)((MObj*)a)->data)[i] = v; }
jobject mock_string(const char* s) {
    MObj* o = mk(K_STRING, (int32_t)strlen(s), 1);
    free(o->data);
    o->data = malloc(strlen(s) + 1);
    memcpy(o->data, s, strlen(s) + 1);
    return (jobject)o;
}
int32_t mock_len(jobject a) { return a ? ((MObj*)a)->len : -1; }
void* mock_data(jobject a) { return a ? ((MObj*)a)->data : NULL; }

/* Pending exception: status of an OmrException, -1 for another class, -2 for none. */
int32_t mock_exception_status(void) {
    if (!g_pending) return -2;
    return strstr(g_pending->name, "OmrException") ? g_pending->status : -1;
}
const char* mock_exception_class(void) { return g_pending ? g_pending->name : ""; }
const char* mock_exception_message(void) { return g_pending ? g_pending->msg : ""; }

/* 0 local refs live, 1 local refs peak, 2 critical-region breaches, 3 pending-exception breaches,
 * 4 null / mistyped argument breaches, 5 critical arrays held now, 6 JNI calls */
int64_t mock_counter(int32_t which) {
    switch (which) {
    case 0: return g_local_live;
    case 1: return g_local_max;
    case 2: return g_crit_violations;
    case 3: return g_exc_violations;
    case 4: return g_arg_violations;
    case 5: return g_crit;
    default: return g_calls;
    }
}

/* Start of a simulated native call: no pending exception, counters cleared (objects kept). */
void mock_begin_call(void) {
    g_pending = NULL;
    g_local_live = g_local_max = 0;
    g_crit_violations = g_exc_violations = g_arg_violations = g_calls = 0;
}

/* Free every object the mock made. */
void mock_reset(void) {
    while (g_all) {
        MObj* n = g_all->next;
        free(g_all->data);
        free(g_all);
        g_all = n;
    }
    g_pending = NULL;
    mock_begin_call();
    g_crit = 0;
}

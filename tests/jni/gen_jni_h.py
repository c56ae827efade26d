#!/usr/bin/env python3
"""Writes tests/jni/jni.h: a TEST-ONLY stand-in for the JDK's jni.h (no JDK in this image) that
declares the JNI types and the JNINativeInterface_ function table in the order the JNI
specification fixes, so jni/omr_jni.c compiles against the mock JVM (tests/jni/mock_jni.c).
Entries the shim never calls are void* slots; the spec's indices are asserted below."""
import os

USED = {
    "GetVersion": "jint (JNICALL *{n})(JNIEnv* env)",
    "FindClass": "jclass (JNICALL *{n})(JNIEnv* env, const char* name)",
    "Throw": "jint (JNICALL *{n})(JNIEnv* env, jthrowable obj)",
    "ThrowNew": "jint (JNICALL *{n})(JNIEnv* env, jclass clazz, const char* msg)",
    "ExceptionOccurred": "jthrowable (JNICALL *{n})(JNIEnv* env)",
    "ExceptionClear": "void (JNICALL *{n})(JNIEnv* env)",
    "DeleteLocalRef": "void (JNICALL *{n})(JNIEnv* env, jobject obj)",
    "NewObject": "jobject (JNICALL *{n})(JNIEnv* env, jclass clazz, jmethodID methodID, ...)",
    "GetMethodID": "jmethodID (JNICALL *{n})(JNIEnv* env, jclass clazz, const char* name, const char* sig)",
    "NewStringUTF": "jstring (JNICALL *{n})(JNIEnv* env, const char* utf)",
    "GetStringUTFChars": "const char* (JNICALL *{n})(JNIEnv* env, jstring str, jboolean* isCopy)",
    "ReleaseStringUTFChars": "void (JNICALL *{n})(JNIEnv* env, jstring str, const char* chars)",
    "GetArrayLength": "jsize (JNICALL *{n})(JNIEnv* env, jarray array)",
    "GetObjectArrayElement": "jobject (JNICALL *{n})(JNIEnv* env, jobjectArray array, jsize index)",
    "NewByteArray": "jbyteArray (JNICALL *{n})(JNIEnv* env, jsize len)",
    "GetByteArrayRegion": "void (JNICALL *{n})(JNIEnv* env, jbyteArray array, jsize start, jsize len, jbyte* buf)",
    "GetIntArrayRegion": "void (JNICALL *{n})(JNIEnv* env, jintArray array, jsize start, jsize len, jint* buf)",
    "GetDoubleArrayRegion": "void (JNICALL *{n})(JNIEnv* env, jdoubleArray array, jsize start, jsize len, "
                            "jdouble* buf)",
    "SetByteArrayRegion": "void (JNICALL *{n})(JNIEnv* env, jbyteArray array, jsize start, jsize len, "
                          "const jbyte* buf)",
    "SetIntArrayRegion": "void (JNICALL *{n})(JNIEnv* env, jintArray array, jsize start, jsize len, const jint* buf)",
    "GetPrimitiveArrayCritical": "void* (JNICALL *{n})(JNIEnv* env, jarray array, jboolean* isCopy)",
    "ReleasePrimitiveArrayCritical": "void (JNICALL *{n})(JNIEnv* env, jarray array, void* carray, jint mode)",
    "ExceptionCheck": "jboolean (JNICALL *{n})(JNIEnv* env)",
}
T = ["Object", "Boolean", "Byte", "Char", "Short", "Int", "Long", "Float", "Double", "Void"]
P = ["Boolean", "Byte", "Char", "Short", "Int", "Long", "Float", "Double"]


def table():
    n = ["reserved0", "reserved1", "reserved2", "reserved3", "GetVersion", "DefineClass", "FindClass",
         "FromReflectedMethod", "FromReflectedField", "ToReflectedMethod", "GetSuperclass", "IsAssignableFrom",
         "ToReflectedField", "Throw", "ThrowNew", "ExceptionOccurred", "ExceptionDescribe", "ExceptionClear",
         "FatalError", "PushLocalFrame", "PopLocalFrame", "NewGlobalRef", "DeleteGlobalRef", "DeleteLocalRef",
         "IsSameObject", "NewLocalRef", "EnsureLocalCapacity", "AllocObject", "NewObject", "NewObjectV",
         "NewObjectA", "GetObjectClass", "IsInstanceOf", "GetMethodID"]
    n += [f"Call{t}Method{s}" for t in T for s in ("", "V", "A")]
    n += [f"CallNonvirtual{t}Method{s}" for t in T for s in ("", "V", "A")]
    n += ["GetFieldID"] + [f"Get{t}Field" for t in T[:9]] + [f"Set{t}Field" for t in T[:9]]
    n += ["GetStaticMethodID"] + [f"CallStatic{t}Method{s}" for t in T for s in ("", "V", "A")]
    n += ["GetStaticFieldID"] + [f"GetStatic{t}Field" for t in T[:9]] + [f"SetStatic{t}Field" for t in T[:9]]
    n += ["NewString", "GetStringLength", "GetStringChars", "ReleaseStringChars", "NewStringUTF",
          "GetStringUTFLength", "GetStringUTFChars", "ReleaseStringUTFChars", "GetArrayLength", "NewObjectArray",
          "GetObjectArrayElement", "SetObjectArrayElement"]
    n += [f"New{t}Array" for t in P] + [f"Get{t}ArrayElements" for t in P] + [f"Release{t}ArrayElements" for t in P]
    n += [f"Get{t}ArrayRegion" for t in P] + [f"Set{t}ArrayRegion" for t in P]
    n += ["RegisterNatives", "UnregisterNatives", "MonitorEnter", "MonitorExit", "GetJavaVM", "GetStringRegion",
          "GetStringUTFRegion", "GetPrimitiveArrayCritical", "ReleasePrimitiveArrayCritical", "GetStringCritical",
          "ReleaseStringCritical", "NewWeakGlobalRef", "DeleteWeakGlobalRef", "ExceptionCheck",
          "NewDirectByteBuffer", "GetDirectBufferAddress", "GetDirectBufferCapacity", "GetObjectRefType", "GetModule"]
    return n


# indices the JNI specification's function table fixes (spot checks; the generator refuses to
# write a table that disagrees)
SPEC_INDEX = {"GetVersion": 4, "FindClass": 6, "Throw": 13, "DeleteLocalRef": 23, "NewObject": 28,
              "GetMethodID": 33, "GetFieldID": 94, "GetStaticMethodID": 113, "GetStaticFieldID": 144,
              "NewStringUTF": 167, "GetArrayLength": 171, "GetObjectArrayElement": 173, "NewByteArray": 176,
              "GetByteArrayRegion": 200, "GetIntArrayRegion": 203, "GetDoubleArrayRegion": 206,
              "SetByteArrayRegion": 208, "SetIntArrayRegion": 211, "RegisterNatives": 215,
              "GetPrimitiveArrayCritical": 222, "ReleasePrimitiveArrayCritical": 223, "ExceptionCheck": 228,
              "GetObjectRefType": 232, "GetModule": 233}


def main():
    names = table()
    assert len(names) == 234, len(names)
    idx = {n: i for i, n in enumerate(names)}
    for n, i in SPEC_INDEX.items():
        assert idx[n] == i, (n, idx[n], i)
    lines = [("    " + USED[n].format(n=n) if n in USED else f"    void* {n}") + f";  /* {i} */"
             for i, n in enumerate(names)]
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "jni.h.in")) as f:
        tmpl = f.read()
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "jni.h"), "w") as f:
        f.write(tmpl.replace("@TABLE@", "\n".join(lines)))


if __name__ == "__main__":
    main()

/*
 * janusgpu_jni.c — JNI shim between org.janusgraph.graphdb.olap.computer.JanusGpu and libjanusgpu's
 * C-ABI (include/janusgpu.h).  Pure pass-through: direct ByteBuffers are handed to the library as
 * raw pointers (no copies), statuses are returned unchanged.  tests/test_jni_shim.py checks that every
 * native method of JanusGpu.java has its function here with the same arity, and
 * tests/test_jni_sequence.py replays GpuGraphComputer's call sequences through ctypes.
 *
 * Build (needs a JDK; none is installed in the build container):
 *   gcc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *       java/native/janusgpu_jni.c -Ljanusgraph_amd -ljanusgpu -Wl,-rpath,'$ORIGIN' -o libjanusgpu_jni.so
 */
#include <jni.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

#include "janusgpu.h"

#define FN(name) Java_org_janusgraph_graphdb_olap_computer_JanusGpu_##name

static void* buf(JNIEnv* env, jobject b) { return b ? (*env)->GetDirectBufferAddress(env, b) : NULL; }

static void put_handle(JNIEnv* env, jlongArray out, const void* h) {
    jlong v = (jlong)(intptr_t)h;
    (*env)->SetLongArrayRegion(env, out, 0, 1, &v);
}

/* Refuse to load against a libjanusgpu whose structs and entry points differ from the header this shim
 * was compiled with (JanusGpu.java checks the same number from the Java side). */
JNIEXPORT jint JNICALL JNI_OnLoad(JavaVM* vm, void* reserved) {
    (void)vm; (void)reserved;
    return jg_abi_version() == JG_ABI_VERSION ? JNI_VERSION_1_8 : JNI_ERR;
}

JNIEXPORT jint JNICALL FN(abiVersion)(JNIEnv* env, jclass c) { (void)env; (void)c; return jg_abi_version(); }

JNIEXPORT jstring JNICALL FN(lastError)(JNIEnv* env, jclass c) {
    (void)c;
    return (*env)->NewStringUTF(env, jg_last_error());
}

JNIEXPORT jint JNICALL FN(ctxCreate)(JNIEnv* env, jclass c, jintArray devices, jlongArray out) {
    (void)c;
    jsize nd = (*env)->GetArrayLength(env, devices);
    jint* d = (*env)->GetIntArrayElements(env, devices, NULL);
    jg_ctx* ctx = NULL;
    int st = jg_ctx_create((const int*)d, (int)nd, &ctx);
    (*env)->ReleaseIntArrayElements(env, devices, d, JNI_ABORT);
    put_handle(env, out, ctx);
    return st;
}

JNIEXPORT jint JNICALL FN(ctxTrim)(JNIEnv* env, jclass c, jlong ctx) {
    (void)env; (void)c;
    return jg_ctx_trim((jg_ctx*)(intptr_t)ctx);
}

JNIEXPORT jint JNICALL FN(ctxDestroy)(JNIEnv* env, jclass c, jlong ctx) {
    (void)env; (void)c;
    return jg_ctx_destroy((jg_ctx*)(intptr_t)ctx);
}

JNIEXPORT jint JNICALL FN(ctxLastStats)(JNIEnv* env, jclass c, jlong ctx, jdoubleArray out9) {
    (void)c;
    jg_stats s;
    int st = jg_ctx_last_stats((const jg_ctx*)(intptr_t)ctx, &s);
    if (st == JG_OK) {
        jdouble v[9] = {s.supersteps, s.levels, s.build_ms, s.compute_ms, s.exchange_ms, s.kernel_ms_total,
                        (jdouble)s.kernel_launches, s.algorithmic_bytes, s.edges_traversed};
        (*env)->SetDoubleArrayRegion(env, out9, 0, 9, v);
    }
    return st;
}

JNIEXPORT jint JNICALL FN(builderCreate)(JNIEnv* env, jclass c, jlong ctx, jlongArray out) {
    (void)c;
    jg_builder* b = NULL;
    int st = jg_builder_create((jg_ctx*)(intptr_t)ctx, &b);
    put_handle(env, out, b);
    return st;
}

JNIEXPORT jint JNICALL FN(builderDestroy)(JNIEnv* env, jclass c, jlong b) {
    (void)env; (void)c;
    return jg_builder_destroy((jg_builder*)(intptr_t)b);
}

JNIEXPORT jint JNICALL FN(builderAddVertices)(JNIEnv* env, jclass c, jlong b, jobject vid, jlong n) {
    (void)c;
    return jg_builder_add_vertices((jg_builder*)(intptr_t)b, (const int64_t*)buf(env, vid), n);
}

JNIEXPORT jint JNICALL FN(builderAddEdges)(JNIEnv* env, jclass c, jlong b, jobject src, jobject dst, jobject weight,
                                           jlong m) {
    (void)c;
    return jg_builder_add_edges((jg_builder*)(intptr_t)b, (const int64_t*)buf(env, src), (const int64_t*)buf(env, dst),
                                (const int32_t*)buf(env, weight), m);
}

JNIEXPORT jint JNICALL FN(builderSetSchema)(JNIEnv* env, jclass c, jlong b, jobject type_ids, jobject type_mult,
                                            jint ntypes, jint partition_bits) {
    (void)c;
    return jg_builder_set_schema((jg_builder*)(intptr_t)b, (const int64_t*)buf(env, type_ids),
                                 (const int8_t*)buf(env, type_mult), ntypes, partition_bits);
}

JNIEXPORT jint JNICALL FN(builderAddRows)(JNIEnv* env, jclass c, jlong b, jobject row_keys, jlong nrows,
                                          jobject row_entry_off, jobject bytes, jlong nbytes, jobject entry_off,
                                          jobject value_pos, jobject entry_weight, jlong nentries) {
    (void)c;
    return jg_builder_add_rows((jg_builder*)(intptr_t)b, (const uint64_t*)buf(env, row_keys), nrows,
                               (const int64_t*)buf(env, row_entry_off), (const uint8_t*)buf(env, bytes), nbytes,
                               (const int64_t*)buf(env, entry_off), (const int32_t*)buf(env, value_pos),
                               (const int32_t*)buf(env, entry_weight), nentries);
}

JNIEXPORT jint JNICALL FN(builderSetWeightKey)(JNIEnv* env, jclass c, jlong b, jlong weight_key, jobject key_ids,
                                               jobject key_types, jint nkeys) {
    (void)c;
    return jg_builder_set_weight_key((jg_builder*)(intptr_t)b, weight_key, (const int64_t*)buf(env, key_ids),
                                     (const int8_t*)buf(env, key_types), nkeys);
}

JNIEXPORT jint JNICALL FN(builderSetQueryLimit)(JNIEnv* env, jclass c, jlong b, jlong limit, jint in_entries) {
    (void)env; (void)c;
    return jg_builder_set_query_limit((jg_builder*)(intptr_t)b, limit, in_entries);
}

JNIEXPORT jint JNICALL FN(builderFinish)(JNIEnv* env, jclass c, jlong b, jint flags, jlongArray out) {
    (void)c;
    jg_graph* g = NULL;
    int st = jg_builder_finish((jg_builder*)(intptr_t)b, (uint32_t)flags, &g);
    put_handle(env, out, g);
    return st;
}

JNIEXPORT jint JNICALL FN(graphDestroy)(JNIEnv* env, jclass c, jlong g) {
    (void)env; (void)c;
    return jg_graph_destroy((jg_graph*)(intptr_t)g);
}

JNIEXPORT jint JNICALL FN(graphInfo)(JNIEnv* env, jclass c, jlong g, jlongArray out8) {
    (void)c;
    jg_graph_info i;
    int st = jg_graph_info_get((const jg_graph*)(intptr_t)g, &i);
    if (st == JG_OK) {
        jlong v[8] = {i.num_vertices, i.num_edges, i.ghost_edges, i.self_loops, i.truncated_vertices,
                      i.max_in_degree, i.max_out_degree, i.device_bytes};
        (*env)->SetLongArrayRegion(env, out8, 0, 8, v);
    }
    return st;
}

JNIEXPORT jint JNICALL FN(graphVertexIds)(JNIEnv* env, jclass c, jlong g, jlong offset, jlong count, jobject vid_out) {
    (void)c;
    return jg_graph_vertex_ids((const jg_graph*)(intptr_t)g, offset, count, (int64_t*)buf(env, vid_out));
}

JNIEXPORT jint JNICALL FN(pageRank)(JNIEnv* env, jclass c, jlong g, jdouble damping, jlong vertex_count,
                                    jint iterations, jobject rank_out, jobject edge_count_out) {
    (void)c;
    return jg_pagerank((jg_graph*)(intptr_t)g, damping, vertex_count, iterations, (double*)buf(env, rank_out),
                       (double*)buf(env, edge_count_out));
}

JNIEXPORT jint JNICALL FN(shortestDistance)(JNIEnv* env, jclass c, jlong g, jlong seed, jint max_depth,
                                            jobject dist_out) {
    (void)c;
    return jg_shortest_distance((jg_graph*)(intptr_t)g, seed, max_depth, (int64_t*)buf(env, dist_out));
}

JNIEXPORT jint JNICALL FN(bfs)(JNIEnv* env, jclass c, jlong g, jobject sources, jint nsrc, jint direction,
                               jint max_depth, jobject depth_out) {
    (void)c;
    return jg_bfs((jg_graph*)(intptr_t)g, (const int64_t*)buf(env, sources), nsrc, direction, max_depth,
                  (int32_t*)buf(env, depth_out));
}

JNIEXPORT jint JNICALL FN(bfsRows)(JNIEnv* env, jclass c, jlong g, jobject sources, jint nsrc, jint direction,
                                   jint max_depth, jobjectArray depth_rows) {
    (void)c;
    if (nsrc <= 0 || (*env)->GetArrayLength(env, depth_rows) < nsrc) return JG_ERR_ARG;
    int32_t** rows = (int32_t**)malloc(sizeof(int32_t*) * (size_t)nsrc);
    if (!rows) return JG_ERR_OOM;
    for (jint s = 0; s < nsrc; ++s) {
        jobject b = (*env)->GetObjectArrayElement(env, depth_rows, s);
        rows[s] = (int32_t*)buf(env, b);
        if (b) (*env)->DeleteLocalRef(env, b);
    }
    int st = jg_bfs_rows((jg_graph*)(intptr_t)g, (const int64_t*)buf(env, sources), nsrc, direction, max_depth, rows);
    free(rows);
    return st;
}

JNIEXPORT jint JNICALL FN(bfsKeep)(JNIEnv* env, jclass c, jlong g, jobject sources, jint nsrc, jint direction,
                                   jint max_depth) {
    (void)c;
    return jg_bfs_keep((jg_graph*)(intptr_t)g, (const int64_t*)buf(env, sources), nsrc, direction, max_depth);
}

JNIEXPORT jint JNICALL FN(bfsKeptRow)(JNIEnv* env, jclass c, jlong g, jint s, jobject depth_out) {
    (void)c;
    return jg_bfs_kept_row((jg_graph*)(intptr_t)g, s, (int32_t*)buf(env, depth_out));
}

JNIEXPORT jint JNICALL FN(bfsKeptRelease)(JNIEnv* env, jclass c, jlong g) {
    (void)env; (void)c;
    return jg_bfs_kept_release((jg_graph*)(intptr_t)g);
}

JNIEXPORT jint JNICALL FN(graphNeighbors)(JNIEnv* env, jclass c, jlong g, jint direction, jobject rows, jlong nrows,
                                          jobject off_out, jobject nbr_out) {
    (void)c;
    return jg_graph_neighbors((const jg_graph*)(intptr_t)g, direction, (const int64_t*)buf(env, rows), nrows,
                              (int64_t*)buf(env, off_out), (int64_t*)buf(env, nbr_out));
}

JNIEXPORT jint JNICALL FN(connectedComponents)(JNIEnv* env, jclass c, jlong g, jobject comp_out,
                                               jintArray iterations_out) {
    (void)c;
    int32_t it = 0;
    int st = jg_connected_components((jg_graph*)(intptr_t)g, (int64_t*)buf(env, comp_out), &it);
    jint v = it;
    (*env)->SetIntArrayRegion(env, iterations_out, 0, 1, &v);
    return st;
}

JNIEXPORT jint JNICALL FN(combineSteps)(JNIEnv* env, jclass c, jlong g, jint direction, jint combiner,
                                        jint int32_wrap, jobject init, jint steps, jobject out, jobject received_out) {
    (void)c;
    return jg_combine_steps((jg_graph*)(intptr_t)g, direction, combiner, int32_wrap, (const int64_t*)buf(env, init),
                            steps, (int64_t*)buf(env, out), (uint8_t*)buf(env, received_out));
}

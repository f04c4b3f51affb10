// Copyright 2026 JanusGraph Authors
// SPDX-License-Identifier: Apache-2.0
package org.janusgraph.graphdb.olap.gpu;

import org.apache.tinkerpop.gremlin.process.computer.Memory;

import java.util.HashMap;
import java.util.Map;
import java.util.Set;

/** Read-only memory of a finished GPU run (FulgoraMemory after complete(), FulgoraMemory.java:97-101). */
final class GpuMemory implements Memory.Admin {
    private final Map<String, Object> map = new HashMap<>();
    private int iteration;
    private long runtime;

    GpuMemory(int iteration, long runtime) {
        this.iteration = iteration;
        this.runtime = runtime;
    }

    void put(String key, Object value) { map.put(key, value); }

    @Override public Set<String> keys() { return map.keySet(); }

    @Override
    @SuppressWarnings("unchecked")
    public <R> R get(String key) {
        final Object r = map.get(key);
        if (r == null) throw Memory.Exceptions.memoryDoesNotExist(key);
        return (R) r;
    }

    @Override public void set(String key, Object value) { map.put(key, value); }
    @Override public void add(String key, Object value) { throw Memory.Exceptions.memoryIsCurrentlyImmutable(); }
    @Override public int getIteration() { return iteration; }
    @Override public long getRuntime() { return runtime; }
    @Override public void setIteration(int i) { iteration = i; }
    @Override public void setRuntime(long r) { runtime = r; }
    @Override public Memory asImmutable() { return this; }
}

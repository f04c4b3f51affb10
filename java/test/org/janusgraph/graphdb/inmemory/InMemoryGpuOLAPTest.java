// Copyright 2026 JanusGraph Authors
// SPDX-License-Identifier: Apache-2.0
package org.janusgraph.graphdb.inmemory;

import org.junit.jupiter.api.AfterAll;
import org.junit.jupiter.api.BeforeAll;

/**
 * The reference's whole OLAPTest suite (janusgraph-backend-testutils/.../olap/OLAPTest.java:89-779) on
 * GpuGraphComputer, with the in-memory configuration of InMemoryOLAPTest (InMemoryOLAPTest.java:30-44).
 * OLAPTest obtains its computer from graph.compute() and withComputer(FulgoraGraphComputer.class); with
 * janusgraph.computer.gpu.default set (java/patches/0001), both return the GPU computer, so every
 * testPageRank / testShortestDistance / testShortestPath / testConnectedComponent / degreeCounting*
 * assertion runs unchanged against it (degree counting through Fulgora's delegate path).
 *
 * Location in the reference tree: janusgraph-inmemory/src/test/java/org/janusgraph/graphdb/inmemory/.
 */
public class InMemoryGpuOLAPTest extends InMemoryOLAPTest {

    private static final String DEFAULT_GPU = "janusgraph.computer.gpu.default";
    private static String previous;

    @BeforeAll
    public static void useGpuComputer() {
        previous = System.getProperty(DEFAULT_GPU);
        System.setProperty(DEFAULT_GPU, "true");
    }

    @AfterAll
    public static void restoreDefaultComputer() {
        if (previous == null) System.clearProperty(DEFAULT_GPU);
        else System.setProperty(DEFAULT_GPU, previous);
    }
}

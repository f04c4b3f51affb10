// Copyright 2026 JanusGraph Authors
// SPDX-License-Identifier: Apache-2.0
package org.janusgraph.graphdb.inmemory;

import org.janusgraph.diskstorage.configuration.BasicConfiguration;
import org.janusgraph.diskstorage.configuration.ModifiableConfiguration;
import org.janusgraph.diskstorage.configuration.WriteConfiguration;
import org.janusgraph.graphdb.configuration.GraphDatabaseConfiguration;

/**
 * The reference's whole OLAPTest suite (janusgraph-backend-testutils/.../olap/OLAPTest.java:89-779) on
 * GpuGraphComputer, with the in-memory configuration of InMemoryOLAPTest (InMemoryOLAPTest.java:30-44).
 * OLAPTest obtains its computer from graph.compute() and withComputer(FulgoraGraphComputer.class); with
 * the graph option computer.gpu.default set (registered and read by java/patches/0001), both return the
 * GPU computer, so every testPageRank / testShortestDistance / testShortestPath / testConnectedComponent /
 * degreeCounting* assertion runs unchanged against it (degree counting through Fulgora's delegate path).
 *
 * Location in the reference tree: janusgraph-inmemory/src/test/java/org/janusgraph/graphdb/inmemory/.
 */
public class InMemoryGpuOLAPTest extends InMemoryOLAPTest {

    @Override
    public WriteConfiguration getConfiguration() {
        final ModifiableConfiguration config = new ModifiableConfiguration(GraphDatabaseConfiguration.ROOT_NS,
            super.getConfiguration(), BasicConfiguration.Restriction.NONE);
        config.set(GraphDatabaseConfiguration.COMPUTER_GPU_DEFAULT, true);
        return config.getConfiguration();
    }
}

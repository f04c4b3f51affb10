// Copyright 2026 JanusGraph Authors
// SPDX-License-Identifier: Apache-2.0
package org.janusgraph.blueprints.inmemory;

import org.apache.tinkerpop.gremlin.GraphProvider;
import org.apache.tinkerpop.gremlin.process.traversal.TraversalStrategy;
import org.apache.tinkerpop.gremlin.process.traversal.dsl.graph.GraphTraversalSource;
import org.apache.tinkerpop.gremlin.structure.Graph;
import org.janusgraph.StorageSetup;
import org.janusgraph.blueprints.AbstractJanusGraphComputerProvider;
import org.janusgraph.diskstorage.configuration.ModifiableConfiguration;
import org.janusgraph.graphdb.configuration.GraphDatabaseConfiguration;
import org.janusgraph.graphdb.olap.computer.GpuGraphComputer;

/**
 * TinkerPop's ProcessComputerSuite against GpuGraphComputer on janusgraph-inmemory: the drop-in criterion
 * of SURVEY §4. The same graph configuration as the Fulgora provider
 * (janusgraph-inmemory/src/test/java/org/janusgraph/blueprints/inmemory/InMemoryGraphComputerProvider.java:27-37,
 * over AbstractJanusGraphComputerProvider.java:28-47), with every computer traversal on the GPU computer.
 * Programs the GPU does not run (TraversalVertexProgram, user programs, graph filters) go to Fulgora inside
 * GpuGraphComputer.submit(), so the suite exercises both paths.
 *
 * Location in the reference tree: janusgraph-inmemory/src/test/java/org/janusgraph/blueprints/inmemory/
 * (INTEGRATION.md). Needs the java/patches and libjanusgpu_jni on java.library.path.
 */
@GraphProvider.Descriptor(computer = GpuGraphComputer.class)
public class InMemoryGpuGraphComputerProvider extends AbstractJanusGraphComputerProvider {

    @Override
    public GraphTraversalSource traversal(final Graph graph) {
        return new GraphTraversalSource(graph).withComputer(GpuGraphComputer.class);
    }

    @Override
    public GraphTraversalSource traversal(final Graph graph, final TraversalStrategy... strategies) {
        return new GraphTraversalSource(graph).withComputer(GpuGraphComputer.class).withStrategies(strategies);
    }

    @Override
    public ModifiableConfiguration getJanusGraphConfiguration(String graphName, Class<?> test, String testMethodName) {
        ModifiableConfiguration config = super.getJanusGraphConfiguration(graphName, test, testMethodName);
        config.setAll(StorageSetup.getInMemoryConfiguration().getAll());
        config.set(GraphDatabaseConfiguration.STORAGE_TRANSACTIONAL, false);
        return config;
    }
}

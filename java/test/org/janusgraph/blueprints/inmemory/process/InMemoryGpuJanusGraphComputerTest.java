// Copyright 2026 JanusGraph Authors
// SPDX-License-Identifier: Apache-2.0
package org.janusgraph.blueprints.inmemory.process;

import org.apache.tinkerpop.gremlin.GraphProviderClass;
import org.apache.tinkerpop.gremlin.process.ProcessComputerSuite;
import org.janusgraph.blueprints.inmemory.InMemoryGpuGraphComputerProvider;
import org.janusgraph.core.JanusGraph;
import org.junit.runner.RunWith;

/**
 * ProcessComputerSuite through GpuGraphComputer, as InMemoryJanusGraphComputerTest runs it through Fulgora
 * (janusgraph-inmemory/src/test/java/org/janusgraph/blueprints/inmemory/process/InMemoryJanusGraphComputerTest.java:23-26).
 * The opt-outs declared on the JanusGraph interface (core/JanusGraph.java:34-62) apply unchanged.
 */
@RunWith(ProcessComputerSuite.class)
@GraphProviderClass(provider = InMemoryGpuGraphComputerProvider.class, graph = JanusGraph.class)
public class InMemoryGpuJanusGraphComputerTest {
}

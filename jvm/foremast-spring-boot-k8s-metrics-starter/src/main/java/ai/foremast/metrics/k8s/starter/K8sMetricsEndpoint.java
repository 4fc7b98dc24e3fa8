package ai.foremast.metrics.k8s.starter;

import org.springframework.boot.actuate.endpoint.annotation.Endpoint;
import org.springframework.boot.actuate.endpoint.annotation.Selector;
import org.springframework.boot.actuate.endpoint.annotation.WriteOperation;

import java.util.Collections;
import java.util.Map;

/**
 * {@code POST /actuator/k8s-metrics/{action}/{metric}} with action enable or
 * disable: flips a meter through the {@link MeterGate} at runtime (when
 * {@code k8s.metrics.enable-common-metrics-filter-action} is on).  Same routes
 * as the Python emitter's {@code /k8s-metrics/{enable,disable}/{metric}}.
 */
@Endpoint(id = "k8s-metrics")
public class K8sMetricsEndpoint {

    private final MeterGate gate;

    public K8sMetricsEndpoint(MeterGate gate) {
        this.gate = gate;
    }

    @WriteOperation
    public Map<String, Object> change(@Selector String action, @Selector String metric) {
        boolean ok;
        if ("enable".equals(action)) {
            ok = gate.enableMetric(metric);
        } else if ("disable".equals(action)) {
            ok = gate.disableMetric(metric);
        } else {
            return Collections.singletonMap("error", "unknown action " + action);
        }
        return Collections.singletonMap(metric, ok ? action + "d" : "filter action disabled");
    }
}

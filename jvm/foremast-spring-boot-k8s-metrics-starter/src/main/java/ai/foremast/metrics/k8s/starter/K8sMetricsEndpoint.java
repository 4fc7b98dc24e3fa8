package ai.foremast.metrics.k8s.starter;

import org.springframework.boot.actuate.endpoint.annotation.Endpoint;
import org.springframework.boot.actuate.endpoint.annotation.ReadOperation;
import org.springframework.boot.actuate.endpoint.annotation.Selector;
import org.springframework.boot.actuate.endpoint.annotation.WriteOperation;

import java.util.Collections;
import java.util.Map;

/**
 * {@code GET /actuator/k8s-metrics/{action}/{metric}} (the reference starter's
 * read operation, so existing callers keep working) and {@code POST} on the
 * same path, with action enable or disable: flips a meter through the
 * {@link MeterGate} at runtime (when
 * {@code k8s.metrics.enable-common-metrics-filter-action} is on).  Same routes
 * as the Python emitter's {@code /k8s-metrics/{enable,disable}/{metric}}.
 */
@Endpoint(id = "k8s-metrics")
public class K8sMetricsEndpoint {

    private final MeterGate gate;

    public K8sMetricsEndpoint(MeterGate gate) {
        this.gate = gate;
    }

    /** GET: the reference's operation (a read operation that toggles). */
    @ReadOperation
    public Map<String, Object> toggle(@Selector String action, @Selector String metric) {
        return change(action, metric);
    }

    @WriteOperation
    public Map<String, Object> change(@Selector String action, @Selector String metric) {
        boolean ok;
        if ("enable".equalsIgnoreCase(action)) {
            ok = gate.enableMetric(metric);
        } else if ("disable".equalsIgnoreCase(action)) {
            ok = gate.disableMetric(metric);
        } else {
            return Collections.singletonMap("error", "unknown action " + action);
        }
        return Collections.singletonMap(metric, ok ? action + "d" : "filter action disabled");
    }
}
